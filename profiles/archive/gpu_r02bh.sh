# r02bh: VALU correlation band height (output rows per workgroup): base 32 vs 16, 24, 48
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base rb16 rb24 rb48 base2; do
  if [ ${v%2} = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --mixed > gpurun_out/r02bh_mix_$v.jsonl 2> gpurun_out/r02bh_mix_$v.err || { tail -5 gpurun_out/r02bh_mix_$v.err; exit 1; }
  timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --ks 3,9,15 > gpurun_out/r02bh_sweep_$v.jsonl 2> gpurun_out/r02bh_sweep_$v.err || { tail -5 gpurun_out/r02bh_sweep_$v.err; exit 1; }
  python - <<PY
import json
print("$v", [(json.loads(l)["k"], json.loads(l)["ms"]) for f in ("mix","sweep") for l in open(f"gpurun_out/r02bh_{f}_$v.jsonl") if l.startswith("{")])
PY
done
