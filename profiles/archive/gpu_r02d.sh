# r02d: NMS tests (strip NMS, rocprim sort) then the full suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "nms or caller or scripted or detect" --timeout 200 --timeout-method thread > gpurun_out/r02d_nms_tests.log 2>&1 || { echo NMS_TESTS_FAILED; tail -40 gpurun_out/r02d_nms_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r02d_nms_tests.log | tail -20
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02d_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02d_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02d_gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02d_bench_B.json 2> gpurun_out/r02d_bench_B.err || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/r02d_bench_B.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_xcorr']['algo'], d['roofline_xcorr']['avg_launch_ms'])
"
