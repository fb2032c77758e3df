# r02au: host-side profile (cProfile) of the config-A module path
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m cProfile -s tottime bench.py --config A --path module --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r02au_module_cprofile.txt 2> gpurun_out/r02au_module.err || exit 1
head -60 gpurun_out/r02au_module_cprofile.txt
