# Round 4: rocprofv3 kernel trace of config E (NMS share of the step)
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_E -o run -- python bench.py --config E --steps 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_E.log 2>&1 || exit 1
python profiles/rocpd_summary.py --label prof_E $O/prof_E > $O/prof_E_kernel_stats.md 2>&1 || true
head -30 $O/prof_E_kernel_stats.md | cut -c1-170
