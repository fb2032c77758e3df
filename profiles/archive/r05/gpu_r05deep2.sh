# Round 5 final tree, deeper random sweep: 5000 + 5000 seeds (the first 1200
# are profiles/r05deep's), per-case worst normwise error logged.
# Run from the repo root: gpurun -- bash profiles/gpu_r05deep2.sh
set -o pipefail
O=gpurun_out/r05deep2
mkdir -p $O
export TMPDIR=/tmp
TMR_RANDOM_SWEEP=5000 timeout -k 10 1000 python -u -m pytest tests/test_gpu_random.py -m gpu -q -s --timeout 900 --timeout-method thread > $O/random_sweep.log 2>&1 || { echo SWEEP_FAILED; grep -E "^FAILED|assert" $O/random_sweep.log | head; tail -5 $O/random_sweep.log; exit 1; }
tail -1 $O/random_sweep.log
