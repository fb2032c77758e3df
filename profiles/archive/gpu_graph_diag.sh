set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 120 python profiles/graph_diag.py > gpurun_out/r04c/graph_diag.log 2>&1; cat gpurun_out/r04c/graph_diag.log | tail -30
