# Round 6 deep checks of the committed tree: the MFMA correlation's random sweep
# (TMR_XCORR_SWEEP seeds), the random detect / module-variant sweeps at 1200 + 1200
# seeds, and every image of the graded batches against the oracle (TMR_FULL_PARITY=1).
# Run from the repo root: gpurun -- bash profiles/gpu_r06_deep.sh <label> [xcorr seeds]
set -o pipefail
L=${1:-r06deep}
N=${2:-400}
O=gpurun_out/$L
mkdir -p $O
export TMPDIR=/tmp
TMR_XCORR_SWEEP=$N timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k random_sweep_vs_oracle --timeout 120 --timeout-method thread > $O/xcorr_sweep.log 2>&1 || { echo XSWEEP_FAILED; tail -30 $O/xcorr_sweep.log; exit 1; }
tail -1 $O/xcorr_sweep.log
TMR_RANDOM_SWEEP=1200 timeout -k 10 400 python -u -m pytest tests/test_gpu_random.py -m gpu -q -s --timeout 350 --timeout-method thread > $O/random_sweep.log 2>&1 || { echo SWEEP_FAILED; tail -30 $O/random_sweep.log; exit 1; }
tail -1 $O/random_sweep.log
TMR_FULL_PARITY=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_headline.py -m gpu -v -k full --timeout 650 --timeout-method thread > $O/full_parity.log 2>&1 || { echo FULL_PARITY_FAILED; tail -30 $O/full_parity.log; exit 1; }
tail -1 $O/full_parity.log
