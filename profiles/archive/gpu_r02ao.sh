# r02ao: halo DMA per-lane offsets hoisted into VGPRs (hoist) vs recomputed per DMA (base)
# base) vs after it (hoist), alternating builds in one call
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base hoist base2 hoist2; do
  if [ ${v%2} = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=${v%2}; fi
  KB_ONLY=split_fp32_heads,split_bf16_heads_acc16,split_fp32_store256_bplane,split_bf16_store256_bplane timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 7 > gpurun_out/r02ao_kb_$v.json 2> gpurun_out/r02ao_kb_$v.err || { tail -5 gpurun_out/r02ao_kb_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02ao_kb_$v.json'));print('$v',{k:v['ms'] for k,v in d.items() if isinstance(v,dict)})"
done
