# r02aa: MFMA correlation 64-row bands on 128-wide maps (libtmr_trb4.so) vs 32-row (this tree): parity of the variant, timings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=trb4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr" > gpurun_out/r02aa_tests.log 2>&1 || { tail -30 gpurun_out/r02aa_tests.log; exit 1; }
tail -1 gpurun_out/r02aa_tests.log
for v in trb2 trb4; do
  if [ $v = trb2 ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --ks 3,5,7,9,11,13,15,21,31 > gpurun_out/r02aa_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --mixed >> gpurun_out/r02aa_kb_$v.jsonl 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import json
for v in ("trb2","trb4"):
    print(v, [(json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02aa_kb_{v}.jsonl") if l.startswith("{")])
PY
