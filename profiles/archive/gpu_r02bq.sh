# r02bq: bench lines of configs D, E and A (detect and module paths) on the current tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config D --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02bq_bench_D.json 2> gpurun_out/r02bq_bench_D.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02bq_bench_E.json 2> gpurun_out/r02bq_bench_E.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02bq_bench_A_detect.json 2> gpurun_out/r02bq_bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02bq_bench_A_module.json 2> gpurun_out/r02bq_bench_A_module.err || exit 1
for c in D E A_detect A_module; do python -c "import json;d=json.load(open('gpurun_out/r02bq_bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'])"; done
