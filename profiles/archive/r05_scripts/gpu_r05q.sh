# Round 5, call q: pixel absmax over channel groups, probability map as a
# chip-wide pass before the peak finder.  Full -m gpu suite; config A detect /
# module against the round-4 tree on this box; kernel traces of A module, B, E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05q.sh
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "TESTS_ABORTED rc=$rc"; tail -30 $O/tests.log; exit 1; }
for t in cur r04 cur; do
  d=.; [ $t != cur ] && d=ab/$t
  (cd $d && timeout -k 10 200 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline) > $O/A_detect_$t.json 2> $O/A_detect_$t.err || { tail -5 $O/A_detect_$t.err; exit 1; }
  (cd $d && timeout -k 10 200 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline) > $O/A_module_$t.json 2> $O/A_module_$t.err || { tail -5 $O/A_module_$t.err; exit 1; }
  for f in A_detect_$t A_module_$t; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_Am -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_Am.log 2>&1 || exit 1
python profiles/rocpd_summary.py $O/prof_Am --label prof_Am > $O/prof_Am_kernel_stats.md 2>&1
for c in B E; do
  timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_$c.log 2>&1 || { echo PROF_FAILED; exit 1; }
  python profiles/rocpd_summary.py $O/prof_$c --label prof_$c > $O/prof_${c}_kernel_stats.md 2>&1
  grep -E "peaks_k|decode_k|prob_k|pixel_absmax" $O/prof_${c}_kernel_stats.md | cut -c1-60,100-200
done
echo done
