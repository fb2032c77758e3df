# PMC passes for configs E and A (profiles/gpu_pmc.sh r04 E A), then the
# config-A host profile (profiles/archive/gpu_r04f.sh).
set -o pipefail
bash profiles/gpu_pmc.sh r04 E A || exit 1
bash profiles/archive/gpu_r04f.sh
