# Round-end check of the committed tree: full -m gpu suite, smoke(), bench B
# (with the CPU baseline) and C, rocprofv3 kernel-trace summary of config B.
# Run from the repo root: gpurun -- bash profiles/gpu_final.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_B.json 2> gpurun_out/bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C --no-cpu-baseline > gpurun_out/bench_C.json 2> gpurun_out/bench_C.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_B -o run -- python bench.py --steps 2 --no-cpu-baseline > gpurun_out/prof_B.log 2>&1 || exit 1
for c in B C; do python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline_xcorr']['hbm_frac'],d['cpu_baseline'])"; done
