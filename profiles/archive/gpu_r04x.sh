# Round 4: rocprofv3 kernel traces of config A (detect: one replayed graph + one sync per image;
# module: the reference's per-exemplar calls) on the final tree
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_A -o run -- python bench.py --config A --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_A.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_A_module -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_A_module.log 2>&1 || exit 1
python profiles/rocpd_summary.py --label prof_A --step-kernel 'split_conv_kernel<3, \d+, 0>' $O/prof_A > $O/prof_A_kernel_stats.md 2>&1 || true
python profiles/rocpd_summary.py --label prof_A_module --step-kernel 'split_conv_kernel<3, \d+, 0>' $O/prof_A_module > $O/prof_A_module_kernel_stats.md 2>&1 || true
tail -8 $O/prof_A_kernel_stats.md; tail -8 $O/prof_A_module_kernel_stats.md
