# r02m: config A module path after the exemplar host-copy memo: module API
# tests, bench line, host-side profile (cProfile)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_headline.py -k "module or demo or trainer" > gpurun_out/r02m_tests.log 2>&1 || exit 1
tail -1 gpurun_out/r02m_tests.log
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02m_bench_A_module.json 2> gpurun_out/r02m_bench_A_module.err || exit 1
timeout -k 10 300 python -m cProfile -o gpurun_out/r02m_amod.prof bench.py --config A --path module --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/r02m_amod.json 2> gpurun_out/r02m_amod.err || exit 1
python - <<'PY'
import json, pstats
d = json.loads(open("gpurun_out/r02m_bench_A_module.json").read().strip().splitlines()[-1])
print("module", d["value"], d["ms_per_step"])
p = pstats.Stats("gpurun_out/r02m_amod.prof")
p.sort_stats("tottime").print_stats(30)
PY
