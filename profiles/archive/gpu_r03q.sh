# r03q: MFMA correlation with the B fragments through a register ring (variant
# libtmr_ring.so, -DTMR_XCORR_BRING=1) -- parity on the variant (MFMA correlation,
# config E, headline tests), then A/B against the current kernel: kbench per k at
# 192^2 / 128^2 (fp32 3-term and bf16 one-term), the config-B and config-E mixes, bench E and B.
# Run from the repo root: gpurun -- bash profiles/gpu_r03q.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=ring timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mfma or config_e or headline or scripted or golden or forward" > gpurun_out/r03q_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03q_tests.log; exit 1; }
tail -1 gpurun_out/r03q_tests.log
for v in main ring; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 3,9,15,17,19,25,31 > gpurun_out/r03q_s192_$v.jsonl 2> gpurun_out/r03q_s192_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 9,19,31 --precision bf16 > gpurun_out/r03q_s192_bf16_$v.jsonl 2> gpurun_out/r03q_s192_bf16_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --ks 5,11,15 > gpurun_out/r03q_s128_$v.jsonl 2> gpurun_out/r03q_s128_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --ks 5,11,15 --precision bf16 > gpurun_out/r03q_s128_bf16_$v.jsonl 2> gpurun_out/r03q_s128_bf16_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 > gpurun_out/r03q_mixE_$v.jsonl 2> gpurun_out/r03q_mixE_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --mixed > gpurun_out/r03q_mixB_$v.jsonl 2> gpurun_out/r03q_mixB_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --algos mfma --mixed --precision bf16 > gpurun_out/r03q_mixC_$v.jsonl 2> gpurun_out/r03q_mixC_$v.err || exit 1
  echo "$v: $(python -c "import json;print([(f,d['k'],d['ms']) for f in ('s192','s192_bf16','s128','s128_bf16','mixE','mixB','mixC') for d in map(json.loads, open('gpurun_out/r03q_'+f+'_$v.jsonl'))])")"
done
for v in main ring main ring; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03q_bench_E_$v.json 2> gpurun_out/r03q_bench_E_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03q_bench_E_$v.json').read().strip().splitlines()[-1]);print('E $v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config B --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03q_bench_B_$v.json 2> gpurun_out/r03q_bench_B_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03q_bench_B_$v.json').read().strip().splitlines()[-1]);print('B $v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
