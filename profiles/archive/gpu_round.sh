# One measurement round: full -m gpu suite, bench B (with CPU baseline) and C,
# rocprofv3 kernel-trace summary of B, PMC HBM-traffic passes (FETCH_SIZE and
# WRITE_SIZE in separate runs, MI355X_MICROARCH.md) for B and C.
# Run from the repo root: gpurun -- bash profiles/gpu_round.sh
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_B.json 2> gpurun_out/bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C --no-cpu-baseline > gpurun_out/bench_C.json 2> gpurun_out/bench_C.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_B -o run -- python bench.py --steps 2 --no-cpu-baseline > gpurun_out/prof_B.log 2>&1 || exit 1
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
python profiles/pmc_assemble.py gpurun_out/pmc "${ROUND:-current}" gpurun_out/decoder_pmc.json > gpurun_out/pmc_assemble.log 2>&1 || exit 1
