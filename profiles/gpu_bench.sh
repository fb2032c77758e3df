# Bench B and C + rocprofv3 kernel-trace summary of config B.
# Run from the repo root: gpurun -- bash profiles/gpu_bench.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_B.json 2> gpurun_out/bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C --no-cpu-baseline > gpurun_out/bench_C.json 2> gpurun_out/bench_C.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_B -o run -- python bench.py --steps 2 --no-cpu-baseline > gpurun_out/prof_B.log 2>&1 || exit 1
