# r02k: split decoder timing experiments (heads launch, 48 units): base vs
# no lo-step weight DMA (1), no halo DMA (2), no step barrier (3) -- the
# variants compute wrong results; they bound what each mechanism costs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base exp1 exp2 exp3; do
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  KB_ONLY=split_fp32_heads,split_fp32_store timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 5 > gpurun_out/r02k_$v.json 2> gpurun_out/r02k_$v.err || exit 1
  echo "$v $(cat gpurun_out/r02k_$v.json)"
done
