# r02ar: decoder step shape (taps per barrier step TPS, weight buffers NWB;
# lookahead NWB-1) -- base: fp32 TPS 2/NWB 2, bf16 TPS 3/NWB 3; variants force
# one precision's shape (bf_* bf16, fp_* fp32)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base bf_t2n4 bf_t4n2 bf_t2n3 fp_t1n3 fp_t1n4 base2; do
  if [ ${v%2} = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  KB_ONLY=split_fp32_heads,split_bf16_heads_acc16,split_fp32_store256_bplane,split_bf16_store256_bplane timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 7 > gpurun_out/r02ar_kb_$v.json 2> gpurun_out/r02ar_kb_$v.err || { tail -5 gpurun_out/r02ar_kb_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02ar_kb_$v.json'));print('$v',{k:v['ms'] for k,v in d.items() if isinstance(v,dict)})"
done
