# r02w: MFMA correlation sweep after the aligned-fragment change, for the
# engine's crossover table (engine.XCORR_COST): 128^2 E=3 every odd k, 192^2 E=16
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python profiles/kbench_xcorr.py --algos mfma,valu --ks 1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31 > gpurun_out/r02w_sweep128.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --algos mfma,valu --images 8 --E 16 --H 192 --ks 3,9,15,21,31 > gpurun_out/r02w_sweep192.jsonl 2>&1 || exit 1
timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma,valu --mixed > gpurun_out/r02w_mixB.jsonl 2>&1 || exit 1
python - <<'PY'
import json
for f in ("r02w_sweep128","r02w_sweep192","r02w_mixB"):
    rows=[json.loads(l) for l in open(f"gpurun_out/{f}.jsonl") if l.startswith("{")]
    for a in ("valu","mfma"):
        print(f, a, [(r["k"], r["ms"]) for r in rows if r["algo"]==a])
PY
