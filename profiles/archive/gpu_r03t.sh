# r03t: A-fragment prefetch distance of the 3-term MFMA correlation at >= 6 tiles per
# wave (192^2: occupancy is LDS-bound, so more rows in flight cost no waves): 1 (main),
# 2 (libtmr_pw2.so), 3 (libtmr_pw3.so) -- MFMA/E tests on each, kbench at 192^2, bench E.
# Run from the repo root: gpurun -- bash profiles/gpu_r03t.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pw2 pw3; do
  TMR_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mfma or config_e" > gpurun_out/r03t_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -30 gpurun_out/r03t_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03t_tests_$v.log)"
done
for v in main pw2 pw3; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 11,15,17,19,25,31 > gpurun_out/r03t_s192_$v.jsonl 2> gpurun_out/r03t_s192_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 > gpurun_out/r03t_mixE_$v.jsonl 2> gpurun_out/r03t_mixE_$v.err || exit 1
  echo "$v: $(python -c "import json;print([(f,d['k'],d['ms']) for f in ('s192','mixE') for d in map(json.loads, open('gpurun_out/r03t_'+f+'_$v.jsonl'))])")"
done
for v in main pw2 pw3 main pw2 pw3; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03t_bench_E_$v.json 2> gpurun_out/r03t_bench_E_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03t_bench_E_$v.json').read().strip().splitlines()[-1]);print('E $v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
