# r02af: one-term MFMA correlation at PF 4: parity, sweep for the cost table, config C bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr or reduced_precision" -s > gpurun_out/r02af_tests.log 2>&1 || { tail -40 gpurun_out/r02af_tests.log; exit 1; }
grep -E "worst normwise|passed|failed" gpurun_out/r02af_tests.log | tail -12
timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --ks 1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31 > gpurun_out/r02af_sweep128_bf16.jsonl 2>&1 || exit 1
timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --images 8 --E 16 --H 192 --ks 3,9,15,21,31 > gpurun_out/r02af_sweep192_bf16.jsonl 2>&1 || exit 1
timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu,mfma --precision bf16 --mixed > gpurun_out/r02af_mixB_bf16.jsonl 2>&1 || exit 1
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02af_bench_C.json 2> gpurun_out/r02af_bench_C.err || { tail -20 gpurun_out/r02af_bench_C.err; exit 1; }
python - <<'PY'
import json
for f in ("sweep128_bf16","sweep192_bf16","mixB_bf16"):
    print(f, [(json.loads(l)["algo"], json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02af_{f}.jsonl") if l.startswith("{")])
d = json.loads(open("gpurun_out/r02af_bench_C.json").read().strip().splitlines()[-1])
x = d["roofline_xcorr"]
print("C", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], x["algo"], x["avg_launch_ms"], json.dumps(x["by_class"]))
PY
