# PMC passes over the VALU correlation kernel (xcorr_rows_kernel; kbench_xcorr,
# config-B shape, k = 3 and k = 15), one counter group per run.
set -o pipefail
mkdir -p gpurun_out/xpmc3
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
for k in 3 15; do
  n=0
  for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/xpmc3/k${k}_p$n -o p -- python profiles/kbench_xcorr.py --ks $k --algos valu --reps 1 > gpurun_out/xpmc3/k${k}_p$n.log 2>&1 || exit 1
  done
  python profiles/pmc_csv.py xcorr_rows gpurun_out/xpmc3/k${k}_p1 gpurun_out/xpmc3/k${k}_p2 gpurun_out/xpmc3/k${k}_p3 gpurun_out/xpmc3/k${k}_p4 > gpurun_out/xpmc3/k${k}_summary.json || exit 1
  cat gpurun_out/xpmc3/k${k}_summary.json
done
