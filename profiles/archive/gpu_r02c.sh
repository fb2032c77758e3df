# r02c: full GPU suite + bench B/E (xcorr cost-model choice) + xcorr sweep (final kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r02c_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02c_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02c_gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02c_bench_B.json 2> gpurun_out/r02c_bench_B.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02c_bench_E.json 2> gpurun_out/r02c_bench_E.err || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --ks 1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31 > gpurun_out/r02c_kbench_sweep128.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --ks 3,9,15,21,31 > gpurun_out/r02c_kbench_sweep192.jsonl 2>&1 || exit 1
python -c "
import json
for f in ['gpurun_out/r02c_bench_B.json','gpurun_out/r02c_bench_E.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['roofline_xcorr']))
"
