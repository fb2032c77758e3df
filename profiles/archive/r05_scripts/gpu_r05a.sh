# Round 5, call a: per-sample / per-pixel activation scales under test
# (precision tests + the parity suite), then a same-box A/B of the round-3
# final, round-4 final and current trees at configs B and E, alternating
# (VERDICT r4 #3).  Ordinary test failures (exit 1) do not stop the A/B;
# a timeout, abort or fault does.
# Run from the repo root: gpurun -- bash profiles/gpu_r05a.sh
set -o pipefail
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
O=gpurun_out/r05a
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
grep -E "^FAILED|worst normwise" $O/tests.log | head -20
[ $rc -le 1 ] || { echo "TESTS_ABORTED rc=$rc"; tail -30 $O/tests.log; exit 1; }
for rep in 1 2; do
  for t in r03 r04 cur; do
    d=.; [ $t != cur ] && d=ab/$t
    for c in B E; do
      (cd $d && timeout -k 10 240 python bench.py --config $c --no-cpu-baseline --no-xcorr-classes) > $O/ab_${t}_${c}_${rep}.json 2> $O/ab_${t}_${c}_${rep}.err || { echo "AB_FAILED $t $c"; tail -20 $O/ab_${t}_${c}_${rep}.err; exit 1; }
      python -c "import json;d=json.load(open('$O/ab_${t}_${c}_${rep}.json'));print('$t $c $rep',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
    done
  done
done
