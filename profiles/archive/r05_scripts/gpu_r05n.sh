# Round 5, call n: final NMS structure (device-wide sort, narrowed windows, batched
# pair loads, CAP 128 lists DMA-staged two blocks ahead, emit kernel); the
# record-output instantiation.  Full -m gpu suite, config E / B kernel
# trace, bench B / C / E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05n.sh
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 160 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "TESTS_ABORTED rc=$rc"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_E -o run -- python bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_E.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof_E.log; exit 1; }
python profiles/rocpd_summary.py $O/prof_E --label prof_E > $O/prof_E_kernel_stats.md 2>&1; head -30 $O/prof_E_kernel_stats.md
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_B -o run -- python bench.py --config B --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_B.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof_B.log; exit 1; }
python profiles/rocpd_summary.py $O/prof_B --label prof_B > $O/prof_B_kernel_stats.md 2>&1; head -30 $O/prof_B_kernel_stats.md
b() {  # b <tag> <args...>
  local tag=$1; shift
  timeout -k 10 170 python bench.py --no-cpu-baseline --no-xcorr-classes "$@" > $O/$tag.json 2> $O/$tag.err || { echo "BENCH_FAILED $tag"; tail -20 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));x=d.get('roofline_xcorr',{});print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],x.get('algo'),x.get('avg_launch_ms'),x.get('hbm_frac'))"
}
for c in B C E; do b ${c} --config $c || exit 1; done
echo done
