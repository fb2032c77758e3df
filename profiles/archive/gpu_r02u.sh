# r02u: MFMA correlation timing-only builds (wrong results): base vs no
# per-row A-fragment global loads (xexp1) vs no B-fragment LDS reads (xexp2)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base xexp3; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --ks 3,15,31 > gpurun_out/r02u_kb_$v.jsonl 2>&1 || exit 1
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --ks 3,9,15 >> gpurun_out/r02u_kb_$v.jsonl 2>&1 || exit 1
done
python - <<'PY'
import json
for v in ("base","xexp3"):
    print(v, [(json.loads(l)["H"], json.loads(l)["k"], json.loads(l)["ms"]) for l in open(f"gpurun_out/r02u_kb_{v}.jsonl") if l.startswith("{")])
PY
