# Round 4: error distribution of the 1,200-case random sweep on the final tree (-s: per-case worst errors)
set -o pipefail
mkdir -p gpurun_out
TMR_RANDOM_SWEEP=600 timeout -k 10 900 python -u -m pytest tests/test_gpu_random.py -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_sweep_errors.log 2>&1 || { tail -20 gpurun_out/r04_sweep_errors.log; exit 1; }
tail -1 gpurun_out/r04_sweep_errors.log
