# Round 6 ablation 2 (temporary TMR_ABL build): 8 = no in-loop band-row LDS reads, 16 = no A-fragment prefetch loads
L=$1; mkdir -p gpurun_out/$L; export TMPDIR=/tmp
K="timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --reps 7"
for a in 0 8 16 24; do
TMR_ABL=$a $K --ks 3,15 > gpurun_out/$L/B_$a.jsonl 2>&1 || exit 1
TMR_ABL=$a $K --images 8 --E 16 --H 192 --ks 31 > gpurun_out/$L/E_$a.jsonl 2>&1 || exit 1
done
for f in gpurun_out/$L/*.jsonl; do echo $f; grep -h '"ms"' $f | python -c "import sys,json;[print(' ',json.loads(l)['k'],json.loads(l)['ms']) for l in sys.stdin]"; done
