# r02bc: one-term bf16 input projection under the bf16 contract; GPU suite, bench B/C
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r02bc_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02bc_tests.log; exit 1; }
tail -1 gpurun_out/r02bc_tests.log
grep "reduced precision" gpurun_out/r02bc_tests.log
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02bc_bench_C.json 2> gpurun_out/r02bc_bench_C.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02bc_bench_B.json 2> gpurun_out/r02bc_bench_B.err || exit 1
for c in B C; do python -c "import json;d=json.load(open('gpurun_out/r02bc_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"; done
