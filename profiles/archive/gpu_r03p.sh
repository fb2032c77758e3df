# r03p: every image of bench.py's configs B, C, D (64 images) and E (8 images)
# against the torch-CPU oracle (tests/test_gpu_headline.py::test_full_batch_every_image).
# Run from the repo root: gpurun --timeout 1150 -- bash profiles/gpu_r03p.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_FULL_PARITY=1 timeout -k 10 1080 python -u -m pytest tests/test_gpu_headline.py -m gpu -k full_batch -x -v -s --timeout 1000 --timeout-method thread > gpurun_out/r03p_full_parity.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03p_full_parity.log; exit 1; }
tail -1 gpurun_out/r03p_full_parity.log
grep -E "worst normwise map error|all .* images" gpurun_out/r03p_full_parity.log
