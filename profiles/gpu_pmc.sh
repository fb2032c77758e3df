# PMC passes (one counter group per run, rocprofv3 --pmc, CSV) over one step of bench.py
# for every config (A-E), one launch per kernel role (--no-xcorr-classes); assembled by
# profiles/pmc_assemble.py into profiles/pmc_by_config.json (bench.py's roofline.traffic).
# Run from the repo root: gpurun -- bash profiles/gpu_pmc.sh <label> [configs...]  (default B C D E A)
set -o pipefail
L=${1:-pmc}
shift
CFGS=${@:-B C D E A}
mkdir -p gpurun_out/pmc_$L
export TMPDIR=/tmp
run() {  # run <name> <bench args> -- <counters...>
    local name=$1; shift; local args=()
    while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$L/$name -o p -- \
        python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-xcorr-classes "${args[@]}" > gpurun_out/pmc_$L/$name.log 2>&1
}
CORE="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_LDS"
for c in $CFGS; do
    run ${c}_fetch --config $c -- FETCH_SIZE || exit 1
    run ${c}_write --config $c -- WRITE_SIZE || exit 1
    run ${c}_core --config $c -- $CORE || exit 1
    echo "config $c done"
done
python profiles/pmc_assemble.py gpurun_out/pmc_$L $L gpurun_out/pmc_$L/pmc_by_config.json > gpurun_out/pmc_$L/assemble.log 2>&1 || { tail -5 gpurun_out/pmc_$L/assemble.log; exit 1; }
cat gpurun_out/pmc_$L/assemble.log
