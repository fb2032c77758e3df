# Round 5 final tree, one call: PMC counters for every config (gpu_pmc.sh),
# then profiles/gpu_r05final.sh (full -m gpu suite, smoke, every bench line,
# kernel traces of B and E, the 2-rank gloo rehearsal).
# Run from the repo root: gpurun -- bash profiles/gpu_r05final2.sh
set -o pipefail
bash profiles/gpu_pmc.sh r05 > gpurun_out/pmc_r05.log 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_r05.log; exit 1; }
tail -1 gpurun_out/pmc_r05.log | cut -c1-200
bash profiles/gpu_r05final.sh r05final2
