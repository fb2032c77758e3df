# PMC passes (one counter group per run, rocprofv3 --pmc, CSV) over one step of
# bench.py config B (fp32 contract) and config C (bf16).
# Run from the repo root: gpurun -- bash profiles/gpu_pmc.sh
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() {  # run <name> <bench args> -- <counters...>
    local name=$1; shift; local args=()
    while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o p -- \
        python bench.py --steps 1 --warmup 0 --no-cpu-baseline "${args[@]}" > gpurun_out/pmc/$name.log 2>&1
}
run B_fetch -- FETCH_SIZE || exit 1
run B_write -- WRITE_SIZE || exit 1
run B_core -- GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS || exit 1
run C_fetch --config C -- FETCH_SIZE || exit 1
run C_write --config C -- WRITE_SIZE || exit 1
run C_core --config C -- GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS || exit 1
