# Round 6: where config A's time goes -- rocprofv3 kernel trace of the detect
# and module paths (graph replay), summarised per kernel and per step (GPU busy
# vs step span) by profiles/rocpd_summary.py.
# Run from the repo root: gpurun -- bash profiles/gpu_r06_alat.sh <label>
set -o pipefail
L=${1:-alat}
O=gpurun_out/$L
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/det -o run -- python bench.py --config A --steps 20 --warmup 3 --no-cpu-baseline > $O/det.json 2> $O/det.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/mod -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline > $O/mod.json 2> $O/mod.err || exit 1
python profiles/rocpd_summary.py $O/det --label A_detect > $O/det.md 2>&1 || exit 1
python profiles/rocpd_summary.py $O/mod --label A_module > $O/mod.md 2>&1 || exit 1
head -40 $O/det.md; head -40 $O/mod.md
