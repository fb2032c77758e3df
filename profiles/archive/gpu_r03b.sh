# r03b: MFMA correlation with whole units per wave (TMR_XCORR_US) -- parity with the
# unit split forced on every shape, then A/B of US=0 vs US=1 (kbench, HIP events) at
# config E's regime (8 x 16 at 192^2) per k and mixed, config B's k>=11 regime, and bench E.
# Run from the repo root: gpurun -- bash profiles/gpu_r03b.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_XCORR_US=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "mfma" --timeout 120 --timeout-method thread > gpurun_out/r03b_us1_tests.log 2>&1 || { echo US1_TESTS_FAILED; tail -30 gpurun_out/r03b_us1_tests.log; exit 1; }
tail -1 gpurun_out/r03b_us1_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q -k "config_e" --timeout 200 --timeout-method thread > gpurun_out/r03b_e_tests.log 2>&1 || { echo E_TEST_FAILED; tail -30 gpurun_out/r03b_e_tests.log; exit 1; }
tail -1 gpurun_out/r03b_e_tests.log
for us in 0 1; do
  TMR_XCORR_US=$us timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 3,9,15,21,31 > gpurun_out/r03b_sweep192_us$us.jsonl 2> gpurun_out/r03b_sweep192_us$us.err || exit 1
  TMR_XCORR_US=$us timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 > gpurun_out/r03b_mixE_us$us.jsonl 2> gpurun_out/r03b_mixE_us$us.err || exit 1
  TMR_XCORR_US=$us timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 --precision bf16 > gpurun_out/r03b_mixE_bf16_us$us.jsonl 2> gpurun_out/r03b_mixE_bf16_us$us.err || exit 1
  TMR_XCORR_US=$us timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --mixed --kmin 11 --kmax 15 > gpurun_out/r03b_mixB11_us$us.jsonl 2> gpurun_out/r03b_mixB11_us$us.err || exit 1
done
for f in sweep192 mixE mixE_bf16 mixB11; do for us in 0 1; do echo "$f us$us: $(python -c "import json;print([(d['k'],d['ms']) for d in map(json.loads, open('gpurun_out/r03b_${f}_us$us.jsonl'))])")"; done; done
timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03b_bench_E.json 2> gpurun_out/r03b_bench_E.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r03b_bench_E.json').read().strip().splitlines()[-1]);print('E',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
