# r02g: reference-exp decode: full GPU suite + smoke + bench B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02g_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02g_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02g_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02g_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/r02g_smoke.log; exit 1; }
cat gpurun_out/r02g_smoke.log | tail -3
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02g_bench_B.json 2> gpurun_out/r02g_bench_B.err || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/r02g_bench_B.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])
"
