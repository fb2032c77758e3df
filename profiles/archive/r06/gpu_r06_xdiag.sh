# Round 6: counters of the window correlation kernel at the config-B mix and
# E k=31 (kbench_xcorr, MFMA only): stall/issue split, MFMA busy, LDS bank
# conflicts, HBM bytes.  One counter pass per run (MI355X_MICROARCH.md).
# Run from the repo root: gpurun -- bash profiles/gpu_r06_xdiag.sh <label>
set -o pipefail
L=${1:-xdiag}
O=gpurun_out/$L
mkdir -p $O
export TMPDIR=/tmp
CORE="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
pass() {  # pass <name> <counters> -- <kbench args>
    local name=$1 ctr=$2; shift 3
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o p -- \
        python profiles/kbench_xcorr.py --algos mfma --reps 3 "$@" > $O/$name.log 2>&1
}
for cfg in B E31; do
    if [ $cfg = B ]; then A="--mixed"; else A="--images 8 --E 16 --H 192 --ks 31"; fi
    pass ${cfg}_core "$CORE" -- $A || exit 1
    pass ${cfg}_fetch FETCH_SIZE -- $A || exit 1
    pass ${cfg}_write WRITE_SIZE -- $A || exit 1
    python profiles/pmc_csv.py xcorr_mfma_kernel $O/${cfg}_core $O/${cfg}_fetch $O/${cfg}_write > $O/${cfg}.json || exit 1
    echo $cfg; cat $O/${cfg}.json
done
