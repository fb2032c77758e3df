# Round-end check of the committed tree: the full -m gpu suite, smoke(), bench lines for every
# config (B with the CPU baseline), and rocprofv3 kernel-trace summaries of configs B and E.
# Run from the repo root: gpurun -- bash profiles/gpu_final.sh <label>
set -o pipefail
L=${1:-final}
O=gpurun_out/$L
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_B.json 2> $O/bench_B.err || exit 1
for c in C D E; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; done
timeout -k 10 300 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline > $O/bench_A_detect.json 2> $O/bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_A_module.json 2> $O/bench_A_module.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_B -o run -- python bench.py --steps 2 --no-cpu-baseline > $O/prof_B.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_E -o run -- python bench.py --config E --steps 2 --no-cpu-baseline > $O/prof_E.log 2>&1 || exit 1
python profiles/rocpd_summary.py $O/prof_B --label prof_B > $O/prof_B_kernel_stats.md || exit 1
python profiles/rocpd_summary.py $O/prof_E --label prof_E > $O/prof_E_kernel_stats.md || exit 1
for c in B C D E A_detect A_module; do python -c "import json;d=json.load(open('$O/bench_$c.json'));x=d['roofline_xcorr'];print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],x['avg_launch_ms'],x['hbm_frac'],x['algo'],d['cpu_baseline'] and d['cpu_baseline']['value'])"; done
