# r02aq: bench lines for configs D, E, A (module + detect) after the decoder
# changes (hoisted halo offsets, packed heads epilogue), rocprof of E
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config D --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02aq_bench_D.json 2> gpurun_out/r02aq_bench_D.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02aq_bench_E.json 2> gpurun_out/r02aq_bench_E.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02aq_bench_A_module.json 2> gpurun_out/r02aq_bench_A_module.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02aq_bench_A_detect.json 2> gpurun_out/r02aq_bench_A_detect.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02aq_E -o run -- python bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02aq_E.log 2>&1 || exit 1
python - <<'PY'
import json
for c in ["D","E","A_module","A_detect"]:
    d=json.loads(open(f"gpurun_out/r02aq_bench_{c}.json").read().strip().splitlines()[-1])
    r=d.get("roofline") or {}
    print(c, d["value"], d["ms_per_step"], r.get("frac"), r.get("executed_frac"), d.get("roofline_xcorr",{}).get("algo"), d.get("roofline_xcorr",{}).get("avg_launch_ms"))
PY
