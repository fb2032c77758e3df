# Round 5, call z: the heads launch's XCD block groups (PXG pixel tiles x NG
# channel tiles per 32 co-resident blocks): 8 x 4 committed vs 4 x 8 / 2 x 16
# (profiles/heads_variants.py pxgN), config E two reps, config B one.
# Run from the repo root: gpurun -- bash profiles/gpu_r05z.sh
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
b() {  # b <tag> <variant> <config>
  if [ $2 = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$2; fi
  timeout -k 10 200 python bench.py --config $3 --no-cpu-baseline --no-xcorr-classes > $O/$1.json 2> $O/$1.err || { echo "BENCH_FAILED $1"; tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
}
for rep in 1 2; do for v in base pxg4 pxg2; do b E_${v}_$rep $v E || exit 1; done; done
for v in base pxg4 pxg2; do b B_$v $v B || exit 1; done
echo done
