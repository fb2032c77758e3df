# r03w: the --gpus launcher at 4 ranks on the 1-GPU box (gloo; every rank on cuda:0),
# the weak-scaling bookkeeping (value = ranks x images / max-over-ranks step time)
# and the per-step all-gather of counts and boxes at world size 4.
# Run from the repo root: gpurun -- bash profiles/gpu_r03w.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --steps 3 --warmup 1 --no-xcorr-classes > gpurun_out/r03w_bench_B_gpus4_gloo.json 2> gpurun_out/r03w_bench_B_gpus4_gloo.err || { tail -20 gpurun_out/r03w_bench_B_gpus4_gloo.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/r03w_bench_B_gpus4_gloo.json') if l.startswith('{')][-1]);print('gpus4 gloo rehearsal', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d['cpu_baseline'])"
