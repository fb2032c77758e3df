# r02i/r02s: VALU correlation kernel variants (old = previous build, new = this tree), parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr" > gpurun_out/r02i_tests.log 2>&1 || exit 1
for v in old new; do
  if [ $v = old ]; then export TMR_LIB_VARIANT=old; else unset TMR_LIB_VARIANT; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --ks 3,5,7,9,11,13,15 > gpurun_out/r02i_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --mixed >> gpurun_out/r02i_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --images 8 --E 16 --H 192 --ks 3,9,15,21,31 >> gpurun_out/r02i_kb_$v.jsonl 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import json
for v in ("old","new"):
    for l in open(f"gpurun_out/r02i_kb_{v}.jsonl"):
        if l.startswith("{"):
            d=json.loads(l); print(v, d.get("H"), d.get("E"), d["k"], d.get("ms"), d.get("valu_frac"), d.get("hbm_frac"))
PY
