# r02b: MFMA correlation kernel: parity tests, then the per-k sweep (VALU vs MFMA) and the config-B mix
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "xcorr" --timeout 120 --timeout-method thread > gpurun_out/r02b_xcorr_tests.log 2>&1 || { echo XCORR_TESTS_FAILED; tail -40 gpurun_out/r02b_xcorr_tests.log; exit 1; }
tail -3 gpurun_out/r02b_xcorr_tests.log
timeout -k 10 300 python profiles/kbench_xcorr.py > gpurun_out/r02b_kbench_sweep128.jsonl 2>&1 || { tail -20 gpurun_out/r02b_kbench_sweep128.jsonl; exit 1; }
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed > gpurun_out/r02b_kbench_mixB.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 > gpurun_out/r02b_kbench_mixE.jsonl 2>&1 || exit 1
cat gpurun_out/r02b_kbench_sweep128.jsonl gpurun_out/r02b_kbench_mixB.jsonl gpurun_out/r02b_kbench_mixE.jsonl
