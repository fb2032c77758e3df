# r03v: NMS reduce with each row block's diagonal words loaded one block ahead (main)
# against the previous kernel (libtmr_old.so): NMS / headline tests, bench E and B, and a
# rocprofv3 kernel trace of config E per arm.
# Run from the repo root: gpurun -- bash profiles/gpu_r03v.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nms or headline or config_e or smoke or golden or demo or trainer" > gpurun_out/r03v_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03v_tests.log; exit 1; }
tail -1 gpurun_out/r03v_tests.log
for v in main old main old; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03v_bench_E_$v.json 2> gpurun_out/r03v_bench_E_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03v_bench_E_$v.json').read().strip().splitlines()[-1]);print('E $v',d['value'],d['ms_per_step'])"
  TMR_LIB_VARIANT=$vv timeout -k 10 300 python bench.py --config B --no-cpu-baseline --no-xcorr-classes > gpurun_out/r03v_bench_B_$v.json 2> gpurun_out/r03v_bench_B_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r03v_bench_B_$v.json').read().strip().splitlines()[-1]);print('B $v',d['value'],d['ms_per_step'])"
done
for v in main old; do
  [ "$v" = main ] && vv="" || vv=$v
  TMR_LIB_VARIANT=$vv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03v_$v -o run -- python bench.py --config E --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03v_$v.log 2>&1 || exit 1
  python profiles/rocpd_summary.py gpurun_out/prof_r03v_$v --label "prof_r03v_$v" > gpurun_out/r03v_E_${v}_kernel_stats.md || exit 1
  echo "$v $(grep -E "strip_kernel" gpurun_out/r03v_E_${v}_kernel_stats.md | cut -c1-50,200-)"
done
