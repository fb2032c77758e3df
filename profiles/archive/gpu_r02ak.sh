# r02ak: heads epilogue A/B in one call (oldepi = r02ag kernel file: scalar
# heads FMAs + xor shuffles; base = v_pk_fma_f32 heads + permlane16/32 swap
# reduce), bf16 acc0 slab (acc16) timing; then the bf16-acc0 engine path:
# GPU suite + config C bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base oldepi base2 oldepi2; do
  if [ ${v%2} = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=${v%2}; fi
  KB_ONLY=split_fp32_heads,split_fp32_heads_noinit,split_bf16_heads,split_bf16_heads_noinit,split_bf16_heads_acc16 timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 7 > gpurun_out/r02ak_kb_$v.json 2> gpurun_out/r02ak_kb_$v.err || { tail -5 gpurun_out/r02ak_kb_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r02ak_kb_$v.json)"
done
unset TMR_LIB_VARIANT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r02ak_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02ak_tests.log; exit 1; }
tail -1 gpurun_out/r02ak_tests.log
grep "reduced precision" gpurun_out/r02ak_tests.log
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02ak_bench_C.json 2> gpurun_out/r02ak_bench_C.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02ak_bench_B.json 2> gpurun_out/r02ak_bench_B.err || exit 1
for c in B C; do python -c "import json;d=json.load(open('gpurun_out/r02ak_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"; done
