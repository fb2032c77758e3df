# r02n: checkpoint -- full GPU suite, smoke, config B and config A (module) bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r02n_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r02n_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02n_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02n_smoke.log 2>&1 || { tail -20 gpurun_out/r02n_smoke.log; exit 1; }
tail -3 gpurun_out/r02n_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02n_bench_B.json 2> gpurun_out/r02n_bench_B.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02n_bench_A_module.json 2> gpurun_out/r02n_bench_A_module.err || exit 1
python - <<'PY'
import json
for c in ["B", "A_module"]:
    d = json.loads(open(f"gpurun_out/r02n_bench_{c}.json").read().strip().splitlines()[-1])
    print(c, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline_xcorr"]["avg_launch_ms"], d.get("cpu_baseline"))
PY
