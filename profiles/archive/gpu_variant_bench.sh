# Bench B per library build variant, interleaved twice (boxes differ in
# clock, so variants are compared inside one call).
# Run from the repo root: gpurun -- bash profiles/gpu_variant_bench.sh <variants...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    [ "$v" = main ] && v=""
    TMR_LIB_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/vb.json 2>/dev/null || exit 1
    echo "variant=${v:-main} $(python -c 'import json;d=json.load(open("gpurun_out/vb.json"));print(d["value"],d["ms_per_step"],d["roofline"]["avg_launch_ms"],d["roofline"]["frac"])')"
  done
done | tee gpurun_out/variant_bench.txt
