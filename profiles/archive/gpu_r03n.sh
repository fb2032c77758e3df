# r03n: two co-resident decoder blocks per CU (variant libtmr_cr2.so: 8 output rows x 32 cols
# x 128 channels per block, 4 waves, <= 80 KB LDS for the 3x3 decoders) -- GPU suite on the
# variant (less the record-layout test, whose torch restatement pads rows to 16),
# variant, then A/B against the one-block-per-CU kernel on bench B, C, E (interleaved).
# Run from the repo root: gpurun -- bash profiles/gpu_r03n.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=cr2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not xpack_records" > gpurun_out/r03n_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03n_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03n_gpu_tests.log
for c in C B E C B E; do for v in main cr2; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03n_bench_${c}_$v.json 2> gpurun_out/r03n_bench_${c}_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03n_bench_${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
done; done
