# r03e: division-free exact IoU test in the NMS mask strips (parity tests + rocprof of
# config E), then the per-config PMC passes (profiles/gpu_pmc.sh) for bench.py's traffic.
# Run from the repo root: gpurun -- bash profiles/gpu_r03e.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "nms or NMS or headline or config_e or pred_boxes or caller or scripted" --timeout 300 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03e_tests.log; exit 1; }
tail -1 gpurun_out/r03e_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03e_E -o run -- python bench.py --config E --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03e_E.log 2>&1 || exit 1
python profiles/rocpd_summary.py gpurun_out/prof_r03e_E | grep -E "strip|sort_boxes"
bash profiles/gpu_pmc.sh r03e
