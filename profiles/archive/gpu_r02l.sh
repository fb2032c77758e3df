# r02l: config A module path timeline (kernel trace) for busy/idle analysis
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_r02l_Amod -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_r02l_Amod.log 2>&1 || exit 1
tail -1 gpurun_out/prof_r02l_Amod.log
