# r03c: row-grouped MFMA correlation (B fragments read once per group of units) and the
# restructured NMS mask strips: full -m gpu suite, MFMA parity with the row-grouped form
# forced on every shape, A/B of TMR_XCORR_RG=0/1 (kbench, HIP events), bench E / C / B.
# Run from the repo root: gpurun -- bash profiles/gpu_r03c.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03c_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03c_gpu_tests.log
TMR_XCORR_RG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "mfma" --timeout 120 --timeout-method thread > gpurun_out/r03c_rg1_tests.log 2>&1 || { echo RG1_TESTS_FAILED; tail -30 gpurun_out/r03c_rg1_tests.log; exit 1; }
tail -1 gpurun_out/r03c_rg1_tests.log
for rg in 0 1; do
  TMR_XCORR_RG=$rg timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 3,9,15,21,31 > gpurun_out/r03c_sweep192_rg$rg.jsonl 2> gpurun_out/r03c_sweep192_rg$rg.err || exit 1
  TMR_XCORR_RG=$rg timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 > gpurun_out/r03c_mixE_rg$rg.jsonl 2> gpurun_out/r03c_mixE_rg$rg.err || exit 1
  TMR_XCORR_RG=$rg timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 --precision bf16 > gpurun_out/r03c_mixE_bf16_rg$rg.jsonl 2> gpurun_out/r03c_mixE_bf16_rg$rg.err || exit 1
  TMR_XCORR_RG=$rg timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --ks 3,7,11,15 > gpurun_out/r03c_sweep128_rg$rg.jsonl 2> gpurun_out/r03c_sweep128_rg$rg.err || exit 1
  TMR_XCORR_RG=$rg timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --mixed > gpurun_out/r03c_mixB_rg$rg.jsonl 2> gpurun_out/r03c_mixB_rg$rg.err || exit 1
  TMR_XCORR_RG=$rg timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --mixed --precision bf16 > gpurun_out/r03c_mixB_bf16_rg$rg.jsonl 2> gpurun_out/r03c_mixB_bf16_rg$rg.err || exit 1
done
timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos valu --mixed > gpurun_out/r03c_mixB_valu.jsonl 2> gpurun_out/r03c_mixB_valu.err || exit 1
for f in sweep192 mixE mixE_bf16 sweep128 mixB mixB_bf16; do for rg in 0 1; do echo "$f rg$rg: $(python -c "import json;print([(d['k'],d['ms']) for d in map(json.loads, open('gpurun_out/r03c_${f}_rg$rg.jsonl'))])")"; done; done
echo "mixB valu: $(python -c "import json;print([(d['k'],d['ms']) for d in map(json.loads, open('gpurun_out/r03c_mixB_valu.jsonl'))])")"
for c in E C B; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03c_bench_$c.json 2> gpurun_out/r03c_bench_$c.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03c_bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline_xcorr']['algo'],d['roofline_xcorr']['avg_launch_ms'],d['roofline_xcorr']['by_class'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03c_E -o run -- python bench.py --config E --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03c_E.log 2>&1 || exit 1
