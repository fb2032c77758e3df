# r02ad: one-term MFMA correlation, A-fragment prefetch distance 1 (this tree) vs 2/4/8 rows (libtmr_pf*.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=pf4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "one_term" > gpurun_out/r02ad_tests.log 2>&1 || { tail -30 gpurun_out/r02ad_tests.log; exit 1; }
tail -1 gpurun_out/r02ad_tests.log
for v in pf1 pf2 pf4 pf8; do
  if [ $v = pf1 ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --ks 3,7,11,15,21,31 > gpurun_out/r02ad_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --mixed >> gpurun_out/r02ad_kb_$v.jsonl 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import json
for v in ("pf1","pf2","pf4","pf8"):
    print(v, [(json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02ad_kb_{v}.jsonl") if l.startswith("{")])
PY
