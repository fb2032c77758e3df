# Round 5, call m: where the NMS greedy wave's time goes at config E --
# rocprof kernel traces of bench E with the committed kernel and with the
# timing-only variants gnolist / gnochain / gnorescan (profiles/heads_variants.py).
# Run from the repo root: gpurun -- bash profiles/gpu_r05m.sh
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
for v in base gnolist gnochain gnorescan; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_$v.log 2>&1 || { echo PROF_FAILED $v; tail -20 $O/prof_$v.log; exit 1; }
  python profiles/rocpd_summary.py $O/prof_$v --label prof_$v > $O/prof_${v}_kernel_stats.md 2>&1
  echo "$v $(grep -E 'greedy_kernel' $O/prof_${v}_kernel_stats.md | cut -c1-60) $(grep -E 'greedy_kernel' $O/prof_${v}_kernel_stats.md | awk -F'|' '{print $5}')"
done
echo done
