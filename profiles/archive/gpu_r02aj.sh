# r02aj: spread acc_init with inline-asm loads (no compiler vmcnt(0) at chunk ends), packed heads epilogue
# chunk) instead of a prologue burst: decoder kbench (48 units) + GPU suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KB_ONLY=split_fp32_heads,split_fp32_heads_noinit,split_bf16_heads,split_bf16_heads_noinit,split_fp32_store,split_bf16_store timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 5 > gpurun_out/r02aj_kb.json 2> gpurun_out/r02aj_kb.err || { tail -5 gpurun_out/r02aj_kb.err; exit 1; }
cat gpurun_out/r02aj_kb.json
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02aj_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02aj_tests.log; exit 1; }
tail -1 gpurun_out/r02aj_tests.log
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02aj_bench_C.json 2> gpurun_out/r02aj_bench_C.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02aj_bench_B.json 2> gpurun_out/r02aj_bench_B.err || exit 1
for c in B C; do python -c "import json;d=json.load(open('gpurun_out/r02aj_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"; done
