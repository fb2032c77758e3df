# Round 5, call g: NMS inputs of configs E and B dumped for the CPU pair
# statistics; config C with the correlation writing the bf16 records vs the
# bf16 plane + record pass (TMR_XCORR_RECORDS), two reps, one lease.
# Run from the repo root: gpurun -- bash profiles/gpu_r05g.sh
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
for c in E B; do
  timeout -k 10 170 python profiles/nms_dump.py --config $c --out $O/nms_$c.npz > $O/dump_$c.log 2>&1 || { echo DUMP_FAILED; tail -20 $O/dump_$c.log; exit 1; }
  cat $O/dump_$c.log
done
b() {  # b <tag> <args...>
  local tag=$1; shift
  timeout -k 10 170 python bench.py --no-cpu-baseline --no-xcorr-classes "$@" > $O/$tag.json 2> $O/$tag.err || { echo "BENCH_FAILED $tag"; tail -20 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));x=d.get('roofline_xcorr',{});print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],x.get('algo'),x.get('avg_launch_ms'),x.get('hbm_frac'))"
}
for rep in 1 2; do
  for r in 1 0; do TMR_XCORR_RECORDS=$r b C_rec${r}_$rep --config C || exit 1; done
done
echo done
