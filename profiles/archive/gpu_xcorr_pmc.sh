# One PMC pass over the correlation kernel (kbench_xcorr, k = 15 and k = 3):
# wave-state counters to see where xcorr_rows_kernel's cycles go.
# Run from the repo root: gpurun -- bash profiles/gpu_xcorr_pmc.sh
set -o pipefail
mkdir -p gpurun_out/xpmc
export TMPDIR=/tmp
for k in 15 3; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/xpmc/k$k -o p -- python profiles/kbench_xcorr.py --kmin $k --kmax $k --reps 1 > gpurun_out/xpmc/k$k.log 2>&1 || exit 1
done
