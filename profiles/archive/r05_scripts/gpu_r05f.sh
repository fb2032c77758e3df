# Round 5, call f: the full -m gpu suite on the tree with the wave-level NMS
# pairs scan, the DMA-staged greedy, the bf16 record output of the
# correlation and the image-major heads order; a kernel trace of config E;
# bench B / C / D / E; the correlation A-fragment source A/B at B and E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05f.sh
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 160 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "TESTS_ABORTED rc=$rc"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_E -o run -- python bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_E.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof_E.log; exit 1; }
python profiles/rocpd_summary.py $O/prof_E --label prof_E > $O/prof_E_kernel_stats.md 2>&1; head -30 $O/prof_E_kernel_stats.md
b() {  # b <tag> <args...>
  local tag=$1; shift
  timeout -k 10 170 python bench.py --no-cpu-baseline --no-xcorr-classes "$@" > $O/$tag.json 2> $O/$tag.err || { echo "BENCH_FAILED $tag"; tail -20 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));x=d.get('roofline_xcorr',{});print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],x.get('algo'),x.get('avg_launch_ms'),x.get('hbm_frac'))"
}
for c in C D; do b ${c} --config $c || exit 1; done
for rep in 1 2; do
  for c in B E; do
    for af in split lds; do TMR_XCORR_AFRAG=$af b ${c}_${af}_$rep --config $c || exit 1; done
  done
done
echo done
