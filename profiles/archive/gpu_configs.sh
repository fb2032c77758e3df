# Full -m gpu suite, bench lines for every BASELINE config that fits one GPU
# (B with the CPU baseline, C, D, E, A) and the rocprofv3 kernel-trace
# summary of config B.  Run from the repo root: gpurun -- bash profiles/gpu_configs.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_B.json 2> gpurun_out/bench_B.err || exit 1
for c in C D E A; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_B -o run -- python bench.py --steps 2 --no-cpu-baseline > gpurun_out/prof_B.log 2>&1 || exit 1
for c in B C D E A; do python -c "import json,sys;d=json.load(open('gpurun_out/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline_xcorr']['hbm_frac'],d['roofline_xcorr']['valu_frac'])"; done
