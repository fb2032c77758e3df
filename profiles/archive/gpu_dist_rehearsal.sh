# Rehearsal of the driver's multi-GPU bench launch on a 1-GPU box: torchrun
# with 1 rank (RCCL path untouched at world 1) and with 2 ranks sharing the
# GPU over gloo (barrier, max-over-ranks timing, all-gather of detections,
# rank-0 JSON).  Run from the repo root: gpurun -- bash profiles/gpu_dist_rehearsal.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dist_n1.json 2> gpurun_out/dist_n1.err || { tail -20 gpurun_out/dist_n1.err; exit 1; }
cat gpurun_out/dist_n1.json
TMR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --batch 16 --no-cpu-baseline > gpurun_out/dist_n2_gloo.json 2> gpurun_out/dist_n2_gloo.err || { tail -20 gpurun_out/dist_n2_gloo.err; exit 1; }
cat gpurun_out/dist_n2_gloo.json
