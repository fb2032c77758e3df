# r02at(b): xpack with a 2-D grid (pixel blocks x, planes y) and 32-bit index math (base)
# math (base) vs the flat 64-bit-index kernel (oldx); then the xpack /
# split-conv GPU tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base oldx base2 oldx2; do
  if [ ${v%2} = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=${v%2}; fi
  KB_ONLY=split_fp32_xpack,split_bf16_xpack timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 7 > gpurun_out/r02at_kb_$v.json 2> gpurun_out/r02at_kb_$v.err || { tail -5 gpurun_out/r02at_kb_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02at_kb_$v.json'));print('$v',{k:v['ms'] for k,v in d.items() if isinstance(v,dict)})"
done
unset TMR_LIB_VARIANT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "split or forward or headline or golden or config" > gpurun_out/r02at_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02at_tests.log; exit 1; }
tail -1 gpurun_out/r02at_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02at_bench_B.json 2> gpurun_out/r02at_bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02at_bench_C.json 2> gpurun_out/r02at_bench_C.err || exit 1
for c in B C; do python -c "import json;d=json.load(open('gpurun_out/r02at_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])"; done
