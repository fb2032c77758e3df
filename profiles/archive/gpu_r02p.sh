# r02p: split decoder with register-staged operand loads (RS) vs the LDS-DMA
# build (libtmr_dma.so, -DTMR_SPLIT_RS=0): parity, kernel timing, config B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py -k "split or heads or golden_forward or forward or headline or config_e" > gpurun_out/r02p_tests.log 2>&1 || { tail -30 gpurun_out/r02p_tests.log; exit 1; }
tail -1 gpurun_out/r02p_tests.log
for v in dma rs; do
  if [ $v = rs ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  KB_ONLY=split_fp32_heads,split_fp32_store,split_bf16_heads timeout -k 10 200 python profiles/kbench_decoder.py --units 48 --reps 5 > gpurun_out/r02p_kb_$v.json 2> gpurun_out/r02p_kb_$v.err || exit 1
  echo "$v $(cat gpurun_out/r02p_kb_$v.json)"
done
unset TMR_LIB_VARIANT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02p_bench_B.json 2> gpurun_out/r02p_bench_B.err || exit 1
TMR_LIB_VARIANT=dma timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02p_bench_B_dma.json 2> gpurun_out/r02p_bench_B_dma.err || exit 1
python - <<'PY'
import json
for c in ["B", "B_dma"]:
    d = json.loads(open(f"gpurun_out/r02p_bench_{c}.json").read().strip().splitlines()[-1])
    print(c, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["executed_frac"])
PY
