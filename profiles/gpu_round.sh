# One GPU round: full -m gpu suite, bench B and C, rocprofv3 kernel trace, PMC traffic passes.
# Run from the repo root: gpurun -- bash profiles/gpu_round.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_B.json 2> gpurun_out/bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C --no-cpu-baseline > gpurun_out/bench_C.json 2> gpurun_out/bench_C.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_B -o run -- python bench.py --steps 2 --no-cpu-baseline > gpurun_out/prof_B.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcB1 -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcB1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcB2 -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcB2.log 2>&1 || exit 1
