# Round 4: one host-input blob per graph + grouped output copies -- GPU suite, config A benches, module trace
set -o pipefail
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
timeout -k 10 300 python bench.py --config A --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_detect$r.json 2> $O/bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_module$r.json 2> $O/bench_A_module.err || exit 1
python -c "import json;[print(n,json.load(open('$O/bench_A_%s$r.json'%n))['ms_per_step']) for n in ('detect','module')]"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_A_module -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_A_module.log 2>&1 || exit 1
python profiles/rocpd_summary.py --label prof_A_module --step-kernel 'split_conv_kernel<3, \d+, 0>' $O/prof_A_module > $O/prof_A_module_kernel_stats.md 2>&1 || true
grep -E "copyBuffer" $O/prof_A_module_kernel_stats.md; tail -5 $O/prof_A_module_kernel_stats.md
