# r02bm: LO3 (F16X3 lo half-chunks in 3-tap steps) variant: split parity
# tests on the variant, kernel microbench and bench B/C, main vs lo3 interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=lo3 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "split or decoder or golden or reduced_precision" > gpurun_out/r02bm_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02bm_tests.log; exit 1; }
tail -1 gpurun_out/r02bm_tests.log
for rep in 1 2; do
  for v in main lo3; do
    [ "$v" = main ] && vv="" || vv=$v
    TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_decoder.py > gpurun_out/r02bm_kb_${v}_${rep}.jsonl 2>&1 || exit 1
  done
done
BENCH_ARGS="--steps 10 --warmup 2" timeout -k 10 600 bash profiles/gpu_variant_bench.sh main lo3 || exit 1
cp gpurun_out/variant_bench.txt gpurun_out/r02bm_variant_B.txt
BENCH_ARGS="--config C --steps 10 --warmup 2" timeout -k 10 600 bash profiles/gpu_variant_bench.sh main lo3 || exit 1
cp gpurun_out/variant_bench.txt gpurun_out/r02bm_variant_C.txt
