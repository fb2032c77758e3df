# r03a: round-3 first check of the tree: full -m gpu suite (incl. the new config C / D
# graded-batch tests), smoke(), bench B (with CPU baseline), C, D, E, rocprofv3 kernel-trace
# of B, and the --gpus 2 launcher rehearsed on one GPU over gloo.
# Run from the repo root: gpurun -- bash profiles/gpu_r03a.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03a_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03a_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03a_gpu_tests.log
grep -E "worst normwise map error|mean kept" gpurun_out/r03a_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03a_smoke.log 2>&1 || { tail -20 gpurun_out/r03a_smoke.log; exit 1; }
tail -1 gpurun_out/r03a_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03a_bench_B.json 2> gpurun_out/r03a_bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C > gpurun_out/r03a_bench_C.json 2> gpurun_out/r03a_bench_C.err || exit 1
timeout -k 10 300 python bench.py --config D --steps 10 --warmup 2 > gpurun_out/r03a_bench_D.json 2> gpurun_out/r03a_bench_D.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 > gpurun_out/r03a_bench_E.json 2> gpurun_out/r03a_bench_E.err || exit 1
for c in B C D E; do python -c "import json;d=json.loads(open('gpurun_out/r03a_bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['path_frac'],d['roofline_xcorr']['dram_min_frac'],d['cpu_baseline'] and d['cpu_baseline']['value'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03a_B -o run -- python bench.py --steps 2 --no-cpu-baseline > gpurun_out/prof_r03a_B.log 2>&1 || exit 1
TMR_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-xcorr-classes > gpurun_out/r03a_bench_B_gpus2_gloo.json 2> gpurun_out/r03a_bench_B_gpus2_gloo.err || { tail -20 gpurun_out/r03a_bench_B_gpus2_gloo.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/r03a_bench_B_gpus2_gloo.json') if l.startswith('{')][-1]);print('gpus2 gloo rehearsal', d['n_gpus'], d['value'], d['config']['parallelism'])"
