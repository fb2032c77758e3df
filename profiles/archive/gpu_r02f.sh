# r02f: module-path reuse + RoIAlign channel groups: full suite, smoke, bench A (module + detect), B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02f_headline.log 2>&1 || { echo HEADLINE_FAILED; tail -40 gpurun_out/r02f_headline.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02f_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02f_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02f_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02f_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/r02f_smoke.log; exit 1; }
timeout -k 10 300 python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02f_bench_A_module.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --config A --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02f_bench_A_detect.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r02f_bench_B.json 2> gpurun_out/r02f_bench_B.err || exit 1
python -c "
import json
for f in ['gpurun_out/r02f_bench_A_module.json','gpurun_out/r02f_bench_A_detect.json','gpurun_out/r02f_bench_B.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'])
"
