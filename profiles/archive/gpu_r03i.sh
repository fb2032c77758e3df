# r03i: persistent heads launch (TMR_SPLIT_PERSIST: one block per CU walks its XCD's tiles;
# the next tile's first halo/weight DMAs go out before this tile's epilogue) -- GPU tests
# with it on, then A/B PERSIST=0/1 on bench B, C, E (interleaved), plus the crossover check.
# Run from the repo root: gpurun -- bash profiles/gpu_r03i.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_SPLIT_PERSIST=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03i_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03i_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03i_gpu_tests.log
for c in B C E B C E; do for g in 0 1; do
  TMR_SPLIT_PERSIST=$g timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03i_bench_${c}_p$g.json 2> gpurun_out/r03i_bench_${c}_p$g.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03i_bench_${c}_p$g.json').read().strip().splitlines()[-1]);x=d['roofline_xcorr'];print('$c p$g',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],x['algo'],x['avg_launch_ms'])"
done; done
