# r03aa: 16-row bands for the 3-term MFMA correlation at >= 192 columns (variant
# libtmr_t1.so: -DTMR_XCORR_TRB1_MINW=192, 50 KB of LDS per block: three blocks per CU
# instead of two; libtmr_t1p.so: the same with 3 rows of A prefetch) -- MFMA/E tests on
# each variant, kbench at 192^2, bench E.
# Run from the repo root: gpurun -- bash profiles/gpu_r03aa.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in t1 t1p; do
  TMR_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mfma or config_e or random" > gpurun_out/r03aa_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -30 gpurun_out/r03aa_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03aa_tests_$v.log)"
done
for v in main t1 t1p; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 11,15,19,25,31 > gpurun_out/r03aa_s192_$v.jsonl 2> gpurun_out/r03aa_s192_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 > gpurun_out/r03aa_mixE_$v.jsonl 2> gpurun_out/r03aa_mixE_$v.err || exit 1
  echo "$v: $(python -c "import json;print([(f,d['k'],d['ms']) for f in ('s192','mixE') for d in map(json.loads, open('gpurun_out/r03aa_'+f+'_$v.jsonl'))])")"
done
for v in main t1 t1p main t1 t1p; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03aa_bench_E_$v.json 2> gpurun_out/r03aa_bench_E_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03aa_bench_E_$v.json').read().strip().splitlines()[-1]);print('E $v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
