# r02v/r02z: MFMA correlation variants (old = previous build, new = this tree): parity, per-k and mixed timings
# the padded-row layout (libtmr_old.so): parity, per-k and mixed timings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py -k "xcorr or config_e" > gpurun_out/r02v_tests.log 2>&1 || { tail -30 gpurun_out/r02v_tests.log; exit 1; }
tail -1 gpurun_out/r02v_tests.log
for v in old new; do
  if [ $v = old ]; then export TMR_LIB_VARIANT=old; else unset TMR_LIB_VARIANT; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --ks 3,5,7,9,11,13,15 > gpurun_out/r02v_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --mixed >> gpurun_out/r02v_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --ks 3,9,15,21,31 >> gpurun_out/r02v_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 >> gpurun_out/r02v_kb_$v.jsonl 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import json
for v in ("old","new"):
    print(v, [(json.loads(l)["H"], json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02v_kb_{v}.jsonl") if l.startswith("{")])
PY
