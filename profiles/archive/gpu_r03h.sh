# r03h: the correlation crossover from the committed rocprof sweep (xcorr_cost.json):
# -m gpu suite, bench B / C / D / E (B picks the MFMA kernel for its mix now).
# Run from the repo root: gpurun -- bash profiles/gpu_r03h.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03h_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03h_gpu_tests.log
for c in B C D E; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03h_bench_$c.json 2> gpurun_out/r03h_bench_$c.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03h_bench_$c.json').read().strip().splitlines()[-1]);x=d['roofline_xcorr'];print('$c',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],x['algo'],x['avg_launch_ms'],{k:(v['algo'],v['avg_launch_ms']) for k,v in x['by_class'].items()})"
done
