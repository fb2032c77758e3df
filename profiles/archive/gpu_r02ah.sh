# r02ah: split decoder heads launch (48 units) -- cost of the acc0 initial
# load (noinit: accumulators from zero), of the heads epilogue (noepi
# build, timing only) and a 4-wave block (nw4 build)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base noepi nw4; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  KB_ONLY=split_fp32_heads,split_fp32_heads_noinit,split_bf16_heads,split_bf16_heads_noinit timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 5 > gpurun_out/r02ah_$v.json 2> gpurun_out/r02ah_$v.err || { tail -5 gpurun_out/r02ah_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r02ah_$v.json)"
done
