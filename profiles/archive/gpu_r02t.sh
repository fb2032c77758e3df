# r02t: MFMA correlation A-fragment prefetch depth on the wide (192-column)
# maps: PF 1 (previous), 2 (this tree), 3; config-E shapes; parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr" > gpurun_out/r02t_tests.log 2>&1 || { tail -20 gpurun_out/r02t_tests.log; exit 1; }
tail -1 gpurun_out/r02t_tests.log
for v in pf1 pf2 pf3; do
  if [ $v = pf2 ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --ks 3,9,15,21,31 > gpurun_out/r02t_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 >> gpurun_out/r02t_kb_$v.jsonl 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import json
for v in ("pf1","pf2","pf3"):
    print(v, [(json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02t_kb_{v}.jsonl") if l.startswith("{")])
PY
