# Round 5, call v: upsample2x output tile rows 32 (committed) / 64 / 128
# (profiles/heads_variants.py uprN), rocprof kernel traces of bench B.
# Run from the repo root: gpurun -- bash profiles/gpu_r05v.sh
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export TMPDIR=/tmp
for v in base upr64 upr128; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --config B --steps 2 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_$v.log 2>&1 || { echo PROF_FAILED $v; tail -20 $O/prof_$v.log; exit 1; }
  python profiles/rocpd_summary.py $O/prof_$v --label prof_$v > $O/prof_${v}_kernel_stats.md 2>&1
  echo "$v $(grep -E 'upsample2x_kernel' $O/prof_${v}_kernel_stats.md | awk -F'|' '{print $3, $5}')"
done
echo done
