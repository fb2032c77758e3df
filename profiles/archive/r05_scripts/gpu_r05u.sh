# Round 5, call u: NMS pairs with one box at a time per wave, lanes over its own window
# (box-broadcast; diag words by atomicOr).  NMS + headline GPU tests, config
# E and B kernel traces, bench E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05u.sh
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -k "nms or NMS or headline or detect" --timeout 160 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "TESTS_ABORTED rc=$rc"; tail -30 $O/tests.log; exit 1; }
for c in E B; do
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_$c.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof_$c.log; exit 1; }
python profiles/rocpd_summary.py $O/prof_$c --label prof_$c > $O/prof_${c}_kernel_stats.md 2>&1; grep -E "greedy|pairs_k|rocprim|bin_|gather_k|sort_boxes" $O/prof_${c}_kernel_stats.md
done
echo done
