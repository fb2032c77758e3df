# r03y (r03x with the half-size rows staged in LDS by the MFMA correlation): fp left at the SAM features' size on the detect path (engine.HalfPlane: RoIAlign
# templates and the MFMA / row-tiled correlation read up2x on the fly; no tmr_upsample2x
# launch): full -m gpu suite (new bit-exactness tests), then bench B / C / E A/B in one call
# (TMR_BENCH_LAZY_UP=0 materialises the plane) and a rocprofv3 kernel trace of B per arm.
# Run from the repo root: gpurun -- bash profiles/gpu_r03y.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03y_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03y_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03y_gpu_tests.log
grep -E "worst normwise map error|mean kept" gpurun_out/r03y_gpu_tests.log
for v in 0 1 0 1; do
  for c in B C; do
    TMR_BENCH_LAZY_UP=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03y_bench_${c}_$v.json 2> gpurun_out/r03y_bench_${c}_$v.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/r03y_bench_${c}_$v.json').read().strip().splitlines()[-1]);print('$c lazy=$v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
  done
done
for v in 0 1; do
  TMR_BENCH_LAZY_UP=1 TMR_BENCH_LAZY_VALU=$v timeout -k 10 300 python bench.py --config D --steps 10 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03y_bench_D_$v.json 2> gpurun_out/r03y_bench_D_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03y_bench_D_$v.json').read().strip().splitlines()[-1]);print('D lazy_valu=$v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
for v in 0 1; do
  TMR_BENCH_LAZY_UP=$v timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03y_bench_E_$v.json 2> gpurun_out/r03y_bench_E_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03y_bench_E_$v.json').read().strip().splitlines()[-1]);print('E lazy=$v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
for v in 0 1; do
  TMR_BENCH_LAZY_UP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03y_B$v -o run -- python bench.py --config B --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03y_B$v.log 2>&1 || exit 1
  python profiles/rocpd_summary.py gpurun_out/prof_r03y_B$v --label "prof_r03y_B$v: TMR_BENCH_LAZY_UP=$v bench.py --config B --steps 2" > gpurun_out/r03y_bench_B${v}_kernel_stats.md || exit 1
done
