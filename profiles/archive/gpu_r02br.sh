# r02br: LDS-transposed record pack for 3-term records at 128- and 256-pixel
# segments (variants t128, t256) vs the one-pixel kernel (main): record test, microbench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TMR_LIB_VARIANT=t256 timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "xpack_records" > gpurun_out/r02br_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02br_tests.log; exit 1; }
tail -1 gpurun_out/r02br_tests.log
for rep in 1 2; do
  for v in main t128 t256; do
    [ "$v" = main ] && vv="" || vv=$v
    TMR_LIB_VARIANT=$vv timeout -k 10 200 python profiles/kbench_decoder.py > gpurun_out/r02br_kb_${v}_${rep}.jsonl 2>&1 || exit 1
    echo "$v $(python -c "import json;d=[json.loads(l) for l in open('gpurun_out/r02br_kb_${v}_${rep}.jsonl') if l.startswith('{')][-1];print(d['split_fp32_xpack']['ms'],d['split_bf16_xpack']['ms'])")"
  done
done
