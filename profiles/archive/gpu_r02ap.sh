# r02ap: halo DMA offsets hoisted (default); GPU suite, bench B/C, rocprof of B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r02ap_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02ap_tests.log; exit 1; }
tail -1 gpurun_out/r02ap_tests.log
grep "reduced precision" gpurun_out/r02ap_tests.log
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02ap_bench_C.json 2> gpurun_out/r02ap_bench_C.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02ap_bench_B.json 2> gpurun_out/r02ap_bench_B.err || exit 1
for c in B C; do python -c "import json;d=json.load(open('gpurun_out/r02ap_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02ap_B -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02ap_B.log 2>&1 || exit 1
