# r02ab: one-term (bf16 / f16) MFMA correlation: parity, then the per-k sweep for the crossover table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr_mfma or reduced_precision" -s > gpurun_out/r02ab_tests.log 2>&1 || { tail -40 gpurun_out/r02ab_tests.log; exit 1; }
grep -E "worst normwise|passed|failed" gpurun_out/r02ab_tests.log | tail -12
timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --ks 1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31 > gpurun_out/r02ab_sweep128_bf16.jsonl 2>&1 || exit 1
timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --images 8 --E 16 --H 192 --ks 3,9,15,21,31 > gpurun_out/r02ab_sweep192_bf16.jsonl 2>&1 || exit 1
timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu,mfma --precision bf16 --mixed > gpurun_out/r02ab_mixB_bf16.jsonl 2>&1 || exit 1
timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision f16 --ks 3,9,15,31 > gpurun_out/r02ab_sweep128_f16.jsonl 2>&1 || exit 1
python - <<'PY'
import json
for f in ("sweep128_bf16","sweep192_bf16","mixB_bf16","sweep128_f16"):
    print(f, [(json.loads(l)["algo"], json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02ab_{f}.jsonl") if l.startswith("{")])
PY
