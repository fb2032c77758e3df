# Round 5, call b: the full -m gpu suite (per-sample scales, ballot peak
# finder, binned NMS, split correlation launch); then A/Bs in one lease:
# correlation split off/on (B, E, C, D, alternating), the image-major heads
# grid variant (launch time + FETCH_SIZE under PMC); a
# rocprof kernel trace of config E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05b.sh
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "TESTS_ABORTED rc=$rc"; tail -30 $O/tests.log; exit 1; }
b() {  # b <tag> <args...>
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-xcorr-classes "$@" > $O/$tag.json 2> $O/$tag.err || { echo "BENCH_FAILED $tag"; tail -20 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));x=d.get('roofline_xcorr',{});print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],x.get('algo'),x.get('avg_launch_ms'),x.get('hbm_frac'))"
}
for rep in 1 2; do
  for c in B E C D; do
    for sp in 0 1; do b ${c}_split${sp}_$rep --config $c --xcorr-split $sp || exit 1; done
  done
done
for rep in 1 2; do
  b B_base_$rep --config B || exit 1
  TMR_LIB_VARIANT=imgmajor b B_imgmajor_$rep --config B || exit 1
done
for v in base imgmajor; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-xcorr-classes --config B > $O/pmc_$v.log 2>&1 || { echo "PMC_FAILED $v"; tail -5 $O/pmc_$v.log; exit 1; }
done
unset TMR_LIB_VARIANT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_E -o run -- python bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_E.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof_E.log; exit 1; }
echo done
