# Round 5, call w: the peak finder stages 16384-pixel chunks (a 128 x 128 map
# at once).  Kernel traces of config A (module path), B and E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05w.sh
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_Am -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_Am.log 2>&1 || exit 1
python profiles/rocpd_summary.py $O/prof_Am --label prof_Am > $O/prof_Am_kernel_stats.md 2>&1
for c in B E; do
  timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/prof_$c.log 2>&1 || { echo PROF_FAILED; exit 1; }
  python profiles/rocpd_summary.py $O/prof_$c --label prof_$c > $O/prof_${c}_kernel_stats.md 2>&1
done
for c in Am B E; do grep -h "peaks_kernel\|prob_kernel\|decode_kernel" $O/prof_${c}_kernel_stats.md | awk -F'|' -v c=$c '{print c, $3, $5, substr($2,1,40)}'; done
