# Round 6 A/B: the correlation's A fragments through a per-block LDS ring (TMR_XCORR_RING=1,
# where two blocks still fit a CU) vs per-wave global loads (0).  Parity first.
L=$1; mkdir -p gpurun_out/$L; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "xcorr or correlation or golden or precision" --timeout 120 --timeout-method thread > gpurun_out/$L/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$L/tests.log
[ $rc -eq 0 ] || { grep -n "Error\|FAILED\|assert" gpurun_out/$L/tests.log | head -20; exit 1; }
K="timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --reps 7"
for r in 0 1; do
export TMR_XCORR_RING=$r
$K --mixed > gpurun_out/$L/B_mix_$r.jsonl 2>&1 && $K --mixed --precision bf16 > gpurun_out/$L/C_mix_$r.jsonl 2>&1 && \
$K --ks 3,9,15 > gpurun_out/$L/B_k_$r.jsonl 2>&1 && \
$K --mixed --images 8 --E 16 --H 192 --kmin 3 --kmax 31 > gpurun_out/$L/E_mix_$r.jsonl 2>&1 || exit 1
done
for f in gpurun_out/$L/*.jsonl; do echo $f; grep -h '"ms"' $f | python -c "import sys,json;[print(' ',json.loads(l)['k'],json.loads(l)['ms'],json.loads(l)['hbm_frac']) for l in sys.stdin]"; done
