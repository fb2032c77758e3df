# Round 5 final tree, deep checks: the random detect / module-variant sweeps
# at 1200 + 1200 seeds (default 200 + 200) with the per-case error log, and
# every image of the graded batches B / C / D / E against the oracle
# (TMR_FULL_PARITY=1).
# Run from the repo root: gpurun -- bash profiles/gpu_r05deep.sh
set -o pipefail
O=gpurun_out/r05deep
mkdir -p $O
export TMPDIR=/tmp
TMR_RANDOM_SWEEP=1200 timeout -k 10 400 python -u -m pytest tests/test_gpu_random.py -m gpu -q -s --timeout 350 --timeout-method thread > $O/random_sweep.log 2>&1 || { echo SWEEP_FAILED; tail -30 $O/random_sweep.log; exit 1; }
tail -1 $O/random_sweep.log
grep -o "worst normwise [0-9.e-]*" $O/random_sweep.log | sort -t' ' -k3 -g | tail -3
TMR_FULL_PARITY=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_headline.py -m gpu -v -k full --timeout 650 --timeout-method thread > $O/full_parity.log 2>&1 || { echo FULL_PARITY_FAILED; tail -30 $O/full_parity.log; exit 1; }
tail -1 $O/full_parity.log
