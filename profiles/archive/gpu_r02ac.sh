# r02ac: config C with the one-term bf16 MFMA correlation; config B unchanged check
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02ac_bench_C.json 2> gpurun_out/r02ac_bench_C.err || { tail -20 gpurun_out/r02ac_bench_C.err; exit 1; }
timeout -k 10 300 python bench.py --config B --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02ac_bench_B.json 2> gpurun_out/r02ac_bench_B.err || { tail -20 gpurun_out/r02ac_bench_B.err; exit 1; }
python - <<'PY'
import json
for c in "CB":
    d = json.loads(open(f"gpurun_out/r02ac_bench_{c}.json").read().strip().splitlines()[-1])
    x = d["roofline_xcorr"]
    print(c, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], x["algo"], x["avg_launch_ms"], json.dumps(x["by_class"]))
PY
