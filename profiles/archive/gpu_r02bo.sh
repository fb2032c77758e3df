# r02bo(b): 4-pixel activation-record pack (xpack4_kernel, per-piece form, no spills): bit-exact record test,
# split/forward tests, kernel microbench and bench B/C, main vs px1 (one-pixel kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "xpack or split or decoder or golden or headline_batch or reduced_precision" > gpurun_out/r02bo3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02bo3_tests.log; exit 1; }
tail -1 gpurun_out/r02bo3_tests.log
for rep in 1 2; do
  for v in main px1; do
    [ "$v" = main ] && vv="" || vv=$v
    TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_decoder.py > gpurun_out/r02bo3_kb_${v}_${rep}.jsonl 2>&1 || exit 1
  done
done
BENCH_ARGS="--steps 10 --warmup 2" timeout -k 10 600 bash profiles/gpu_variant_bench.sh main px1 || exit 1
cp gpurun_out/variant_bench.txt gpurun_out/r02bo3_variant_B.txt
BENCH_ARGS="--config C --steps 10 --warmup 2" timeout -k 10 600 bash profiles/gpu_variant_bench.sh main px1 || exit 1
cp gpurun_out/variant_bench.txt gpurun_out/r02bo3_variant_C.txt
