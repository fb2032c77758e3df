# Round 4: every image of the B/C/D/E bench batches against the oracle on the final kernels (6-bit hi weights)
set -o pipefail
mkdir -p gpurun_out
TMR_FULL_PARITY=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py -m gpu -k full_batch -x -v -s --timeout 800 --timeout-method thread > gpurun_out/${1:-r04q}_full_parity.log 2>&1 || { echo FULL_PARITY_FAILED; tail -40 gpurun_out/${1:-r04q}_full_parity.log; exit 1; }
tail -3 gpurun_out/${1:-r04q}_full_parity.log
