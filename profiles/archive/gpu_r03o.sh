# r03o: MFMA correlation with the second K block of w >= 19 templates on 16x16x16 MFMAs
# (variant libtmr_k48.so: K 64 -> 48) -- parity on the variant (all MFMA correlation tests,
# config E), then A/B against the current kernel: kbench per k and config-E mix, bench E.
# Run from the repo root: gpurun -- bash profiles/gpu_r03o.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=k48 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "mfma or config_e or headline or scripted or golden or forward" > gpurun_out/r03o_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03o_tests.log; exit 1; }
tail -1 gpurun_out/r03o_tests.log
grep -E "xcorr mfma" gpurun_out/r03o_tests.log | head -20
for v in main k48; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 15,17,19,21,25,31 > gpurun_out/r03o_sweep192_$v.jsonl 2> gpurun_out/r03o_sweep192_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --ks 19,25,31 --precision bf16 > gpurun_out/r03o_sweep192_bf16_$v.jsonl 2> gpurun_out/r03o_sweep192_bf16_$v.err || exit 1
  TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --algos mfma --mixed --kmin 3 --kmax 31 > gpurun_out/r03o_mixE_$v.jsonl 2> gpurun_out/r03o_mixE_$v.err || exit 1
  echo "$v: $(python -c "import json;print([(d['k'],d['ms']) for f in ('sweep192','sweep192_bf16','mixE') for d in map(json.loads, open('gpurun_out/r03o_'+f+'_$v.jsonl'))])")"
done
for v in main k48 main k48; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03o_bench_E_$v.json 2> gpurun_out/r03o_bench_E_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03o_bench_E_$v.json').read().strip().splitlines()[-1]);print('E $v',d['value'],d['ms_per_step'],d['roofline_xcorr']['avg_launch_ms'])"
done
