# r03r: the bf16 contract's f_TM as a bf16 plane (tmr_xcorr_out + tmr_split_xpack16):
# full -m gpu suite (new: xcorr_out / xpack16 bit-exactness, engine bit-identity with the
# fp32 plane), then bench C A/B in one call (TMR_BENCH_OUT_BF16=0 keeps the fp32 plane)
# with a rocprofv3 kernel trace of each arm.
# Run from the repo root: gpurun -- bash profiles/gpu_r03r.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03r_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03r_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03r_gpu_tests.log
grep -E "worst normwise map error|mean kept" gpurun_out/r03r_gpu_tests.log
for v in 0 1 0 1; do
  TMR_BENCH_OUT_BF16=$v timeout -k 10 300 python bench.py --config C --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03r_bench_C_$v.json 2> gpurun_out/r03r_bench_C_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03r_bench_C_$v.json').read().strip().splitlines()[-1]);print('C out_bf16=$v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
for v in 0 1; do
  TMR_BENCH_OUT_BF16=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03r_C$v -o run -- python bench.py --config C --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03r_C$v.log 2>&1 || exit 1
  python profiles/rocpd_summary.py gpurun_out/prof_r03r_C$v --label "prof_r03r_C$v: TMR_BENCH_OUT_BF16=$v bench.py --config C --steps 2" > gpurun_out/r03r_bench_C${v}_kernel_stats.md || exit 1
  grep -E "xcorr|xpack" gpurun_out/r03r_bench_C${v}_kernel_stats.md | cut -c1-60,200-
done
