# r02e: rocprofv3 kernel-trace stats for bench config B (detect path) and
# config A on the module path (demo.py call sequence)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02e_B -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02e_B.log 2>&1 || { tail -20 gpurun_out/prof_r02e_B.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02e_Amod -o run -- python bench.py --config A --path module --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r02e_Amod.log 2>&1 || { tail -20 gpurun_out/prof_r02e_Amod.log; exit 1; }
ls -R gpurun_out/prof_r02e_B | head -20
