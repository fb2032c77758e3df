# r03m: no activation-scale reductions under the bf16 contract (bf16 records and kernels are
# unscaled): full -m gpu suite, bench C twice.
# Run from the repo root: gpurun -- bash profiles/gpu_r03m.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03m_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03m_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03m_gpu_tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03m_bench_C_$r.json 2> gpurun_out/r03m_bench_C_$r.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03m_bench_C_$r.json').read().strip().splitlines()[-1]);print('C',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
