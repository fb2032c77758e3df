# Round 4: the default -m gpu suite on the final tree (random sweep now 200 + 200)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_final_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04_final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04_final_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final_smoke.log 2>&1 || { tail -20 gpurun_out/r04_final_smoke.log; exit 1; }
head -1 gpurun_out/r04_final_smoke.log
