# r03f: heads launch with an image's units innermost in the block order
# (TMR_SPLIT_UNITS_PER_IMAGE) and the 4-wave NMS mask strips: full -m gpu suite, then A/B of
# TMR_SPLIT_GROUP_UNITS=0/1 on bench B, C, E (interleaved), heads launch times from the lines.
# Run from the repo root: gpurun -- bash profiles/gpu_r03f.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03f_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03f_gpu_tests.log
for c in B C E B C E; do for g in 0 1; do
  TMR_SPLIT_GROUP_UNITS=$g timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03f_bench_${c}_g$g.json 2> gpurun_out/r03f_bench_${c}_g$g.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03f_bench_${c}_g$g.json').read().strip().splitlines()[-1]);print('$c g$g',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
done; done
