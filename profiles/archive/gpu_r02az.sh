# r02az: VALU correlation with two output rows' FMA chains interleaved per
# tap (base) vs one row at a time (oldxc): per-k sweep at 128^2 E=3, the
# config-B mix; then the xcorr GPU tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base oldxc; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --ks 3,5,7,9,11,13,15,21,31 > gpurun_out/r02az_sweep_$v.jsonl 2> gpurun_out/r02az_sweep_$v.err || { tail -5 gpurun_out/r02az_sweep_$v.err; exit 1; }
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --mixed > gpurun_out/r02az_mix_$v.jsonl 2> gpurun_out/r02az_mix_$v.err || { tail -5 gpurun_out/r02az_mix_$v.err; exit 1; }
  python - <<PY
import json
for f in ("sweep","mix"):
    print("$v", f, [(json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02az_{f}_$v.jsonl") if l.startswith("{")])
PY
done
unset TMR_LIB_VARIANT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "xcorr or golden or headline" > gpurun_out/r02az_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02az_tests.log; exit 1; }
tail -1 gpurun_out/r02az_tests.log
