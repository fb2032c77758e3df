# Round 4: a deep randomized parity sweep on the final tree (600 detect configs + 300 module variants)
set -o pipefail
mkdir -p gpurun_out
TMR_RANDOM_SWEEP=${1:-600} timeout -k 10 1000 python -u -m pytest tests/test_gpu_random.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_random_sweep.log 2>&1 || { echo SWEEP_FAILED; tail -30 gpurun_out/r04_random_sweep.log; exit 1; }
tail -2 gpurun_out/r04_random_sweep.log
