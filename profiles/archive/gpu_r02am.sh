# r02am: heads with the engine's acc0 sharing (3 units per image slab) vs a
# slab per unit, and the fp-half store at K = 256 with / without the
# broadcast bias-plane initial values
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 2; do
KB_ONLY=split_fp32_heads,split_fp32_heads_e3,split_fp32_heads_noinit,split_bf16_heads_acc16,split_bf16_heads_e3,split_bf16_heads_noinit,split_fp32_store256_bplane,split_fp32_store256_noinit,split_bf16_store256_bplane,split_bf16_store256_noinit timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 7 > gpurun_out/r02am_kb$v.json 2> gpurun_out/r02am_kb$v.err || { tail -5 gpurun_out/r02am_kb$v.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02am_kb$v.json'));print({k:v['ms'] for k,v in d.items() if isinstance(v,dict)})"
done
