# r03d: NMS mask strips (4 waves x 8 column blocks per block, row-contiguous stores) --
# NMS parity tests, then rocprof of config E with the new strips and with the previous
# kernel (libtmr_nmsold.so, TMR_LIB_VARIANT), and rocprof of config C (its step breakdown).
# Run from the repo root: gpurun -- bash profiles/gpu_r03d.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "nms or NMS or headline or config_e or smoke" --timeout 300 --timeout-method thread > gpurun_out/r03d_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03d_tests.log; exit 1; }
tail -1 gpurun_out/r03d_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03d_E -o run -- python bench.py --config E --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03d_E.log 2>&1 || exit 1
TMR_LIB_VARIANT=nmsold timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03d_E_nmsold -o run -- python bench.py --config E --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03d_E_nmsold.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03d_C -o run -- python bench.py --config C --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03d_C.log 2>&1 || exit 1
python profiles/rocpd_summary.py gpurun_out/prof_r03d_E | grep -E "strip|sort_boxes"
python profiles/rocpd_summary.py gpurun_out/prof_r03d_E_nmsold | grep -E "strip|sort_boxes"
