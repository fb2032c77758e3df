L=$1; mkdir -p gpurun_out/$L; export TMPDIR=/tmp
K="timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --reps 7"
for a in 0 1 2 3 4 5 7; do
TMR_ABL=$a $K --ks 3,15 > gpurun_out/$L/B_$a.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python profiles/kbench_xcorr.py --algos valu --reps 7 --ks 3,15 > gpurun_out/$L/B_valu.jsonl 2>&1 || exit 1
for f in gpurun_out/$L/*.jsonl; do echo $f; grep -h '"ms"' $f | python -c "import sys,json;[print(' ',json.loads(l)['k'],json.loads(l)['ms']) for l in sys.stdin]"; done
