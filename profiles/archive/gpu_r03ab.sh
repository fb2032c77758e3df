# r03ab: XCD block-group shape of the decoder heads launch (pixel tiles x channel tiles per
# XCD wave of 32 blocks): 8 x 4 (main), 16 x 2 (p16), 4 x 8 (p4), 32 x 1 (p32) -- headline
# tests on each, bench B and C, and a FETCH_SIZE pass of config B's heads launch per arm.
# Run from the repo root: gpurun -- bash profiles/gpu_r03ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in p16 p4 p32; do
  TMR_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "headline_batch_config_b or split or random_config" > gpurun_out/r03ab_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -30 gpurun_out/r03ab_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03ab_tests_$v.log)"
done
for v in main p16 p4 p32 main p16 p4 p32; do
  [ "$v" = main ] && vv="" || vv=$v
  for c in B C; do
    TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03ab_bench_${c}_$v.json 2> gpurun_out/r03ab_bench_${c}_$v.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/r03ab_bench_${c}_$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c $v',d['value'],d['ms_per_step'],r['avg_launch_ms'])"
  done
done
for v in main p16 p4 p32; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03ab_fetch_$v -o p -- python bench.py --config B --steps 1 --warmup 0 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03ab_fetch_$v.log 2>&1 || exit 1
  python profiles/pmc_csv.py 'split_conv_kernel<\d+, \d+, 1>' gpurun_out/r03ab_fetch_$v > gpurun_out/r03ab_fetch_$v.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r03ab_fetch_$v.json'));print('B heads FETCH $v', d['counters']['FETCH_SIZE'])"
done
