L=$1; mkdir -p gpurun_out/$L; export TMPDIR=/tmp
K="timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --reps 7"
for br in 32 64; do
export TMR_XCORR_BR_EXPERIMENT=$br
$K --mixed > gpurun_out/$L/B_mix_$br.jsonl 2>&1 && $K --mixed --precision bf16 > gpurun_out/$L/C_mix_$br.jsonl 2>&1 && \
$K --ks 3,9,15 > gpurun_out/$L/B_k_$br.jsonl 2>&1 && \
$K --images 8 --E 16 --H 192 --ks 3,11,15,31 > gpurun_out/$L/E_k_$br.jsonl 2>&1 || exit 1
done
for f in gpurun_out/$L/*.jsonl; do echo $f; grep -h '"ms"' $f | python -c "import sys,json;[print(' ',json.loads(l)['k'],json.loads(l)['ms']) for l in sys.stdin]"; done
