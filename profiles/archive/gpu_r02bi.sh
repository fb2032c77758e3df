# r02bi: NMS IoU test without the fp32 division (exact rational comparison);
# full GPU suite, bench E / B, rocprof of E
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02bi_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02bi_tests.log; exit 1; }
tail -1 gpurun_out/r02bi_tests.log
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02bi_bench_E.json 2> gpurun_out/r02bi_bench_E.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02bi_bench_B.json 2> gpurun_out/r02bi_bench_B.err || exit 1
for c in E B; do python -c "import json;d=json.load(open('gpurun_out/r02bi_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02bi_E -o run -- python bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02bi_E.log 2>&1 || exit 1
