# r03z: full -m gpu suite on the tree after the r03x/r03y revert (one-term template split
# writing the hi fragments only) + bench C.
# Run from the repo root: gpurun -- bash profiles/gpu_r03z.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03z_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03z_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03z_gpu_tests.log
timeout -k 10 300 python bench.py --config C --no-cpu-baseline > gpurun_out/r03z_bench_C.json 2> gpurun_out/r03z_bench_C.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r03z_bench_C.json').read().strip().splitlines()[-1]);print('C',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
