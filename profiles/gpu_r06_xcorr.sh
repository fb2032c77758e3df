# Round 6: the 2-D window Toeplitz correlation -- its parity tests, then
# per-k and mixed launch times at configs B (128^2, E = 3), C (bf16) and E
# (192^2, E = 16).  Run from the repo root: gpurun -- bash profiles/gpu_r06_xcorr.sh [label]
L=${1:-r06f}
mkdir -p gpurun_out/$L
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "xcorr or correlation or golden or precision" --timeout 120 --timeout-method thread > gpurun_out/$L/tests.log 2>&1; rc=$?
tail -2 gpurun_out/$L/tests.log
[ $rc -eq 0 ] || { grep -n "Error\|FAILED\|assert" gpurun_out/$L/tests.log | head -20; exit 1; }
K="timeout -k 10 200 python profiles/kbench_xcorr.py --algos mfma --reps 7"
$K --mixed > gpurun_out/$L/B_mix.jsonl 2>&1 && $K --mixed --precision bf16 > gpurun_out/$L/C_mix.jsonl 2>&1 && \
$K --mixed --images 8 --E 16 --H 192 --kmin 3 --kmax 31 > gpurun_out/$L/E_mix.jsonl 2>&1 && \
$K --ks 3,5,7,9,11,13,15 > gpurun_out/$L/B_k.jsonl 2>&1 && \
$K --images 8 --E 16 --H 192 --ks 3,7,11,15,19,23,27,31 > gpurun_out/$L/E_k.jsonl 2>&1 || exit 1
for f in gpurun_out/$L/*.jsonl; do echo $f; grep -h '"ms"' $f | python -c "import sys,json;[print(' ',json.loads(l)['k'],json.loads(l)['ms'],json.loads(l)['hbm_frac']) for l in sys.stdin]"; done
