# r03s: rows per block of the bf16-input record pack (tmr_split_xpack16): 4 (main),
# 1 (libtmr_r1.so), 8 (libtmr_r8.so) -- record bit-exactness on each, then bench C
# and a rocprofv3 kernel trace per arm.
# Run from the repo root: gpurun -- bash profiles/gpu_r03s.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in main r1 r8; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xpack or bf16_ftm or config_c or one_term" > gpurun_out/r03s_tests_$v.log 2>&1 || { echo TESTS_FAILED $v; tail -30 gpurun_out/r03s_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03s_tests_$v.log)"
done
for v in main r1 r8 main r1 r8; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config C --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03s_bench_C_$v.json 2> gpurun_out/r03s_bench_C_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03s_bench_C_$v.json').read().strip().splitlines()[-1]);print('C $v',d['value'],d['ms_per_step'])"
done
for v in main r1 r8; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03s_$v -o run -- python bench.py --config C --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03s_$v.log 2>&1 || exit 1
  python profiles/rocpd_summary.py gpurun_out/prof_r03s_$v --label "prof_r03s_$v" > gpurun_out/r03s_C_${v}_kernel_stats.md || exit 1
  echo "$v $(grep -E "xpack4" gpurun_out/r03s_C_${v}_kernel_stats.md | cut -c1-40,190-)"
done
