# r02ae: A-fragment prefetch distance: one-term PF 3/4/5 (libtmr_pf*.so), 3-term PF 1 (tree) / 2 / 4 (libtmr_s*.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=s4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr_mfma_vs" > gpurun_out/r02ae_tests.log 2>&1 || { tail -30 gpurun_out/r02ae_tests.log; exit 1; }
tail -1 gpurun_out/r02ae_tests.log
for v in pf3 pf4 pf5; do
  export TMR_LIB_VARIANT=$v
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --ks 3,7,11,15,21,31 > gpurun_out/r02ae_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --precision bf16 --mixed >> gpurun_out/r02ae_kb_$v.jsonl 2>&1 || exit 1
done
for v in s1 s2 s4; do
  if [ $v = s1 ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --ks 3,7,11,15,21,31 > gpurun_out/r02ae_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --mixed >> gpurun_out/r02ae_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --ks 3,15,31 >> gpurun_out/r02ae_kb_$v.jsonl 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import json
for v in ("pf3","pf4","pf5","s1","s2","s4"):
    print(v, [(json.loads(l)["H"], json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02ae_kb_{v}.jsonl") if l.startswith("{")])
PY
