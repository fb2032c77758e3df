L=$1; mkdir -p gpurun_out/$L; export TMPDIR=/tmp
K="timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --reps 7"
for ua in 4 8; do
export TMR_XCORR_UA=$ua
$K --mixed > gpurun_out/$L/B_mix_$ua.jsonl 2>&1 && $K --mixed --precision bf16 > gpurun_out/$L/C_mix_$ua.jsonl 2>&1 && \
$K --ks 3,15 > gpurun_out/$L/B_k_$ua.jsonl 2>&1 && \
$K --images 8 --E 16 --H 192 --ks 7,31 > gpurun_out/$L/E_k_$ua.jsonl 2>&1 && \
$K --mixed --images 8 --E 16 --H 192 --kmin 3 --kmax 31 > gpurun_out/$L/E_mix_$ua.jsonl 2>&1 || exit 1
done
for f in gpurun_out/$L/*.jsonl; do echo $f; grep -h '"ms"' $f | python -c "import sys,json;[print(' ',json.loads(l)['k'],json.loads(l)['ms']) for l in sys.stdin]"; done
