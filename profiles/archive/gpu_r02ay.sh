# r02ay: XCD block-group shape of the decoder kernel (pixel tiles x channel
# tiles per 32-block XCD round) re-measured: base 8x4 vs 16x2, 4x8, 32x1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base g16x2 g4x8 g32x1 base2; do
  if [ ${v%2} = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  KB_ONLY=split_fp32_heads_e3,split_bf16_heads_e3,split_fp32_store256_bplane timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 7 > gpurun_out/r02ay_kb_$v.json 2> gpurun_out/r02ay_kb_$v.err || { tail -5 gpurun_out/r02ay_kb_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02ay_kb_$v.json'));print('$v',{k:v['ms'] for k,v in d.items() if isinstance(v,dict)})"
done
