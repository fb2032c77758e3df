# Round 4: the 6-bit hi weights fail the 1e-5 contract on one random module variant (seed 188: k = 1,
# 16 channels, b map 1.33e-5). The same case at 8 and 11 bits, then the deep sweep at 8 bits.
set -o pipefail
O=gpurun_out/r04wb
mkdir -p $O
for v in base wsparse8 wsparse11; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR TMR_RANDOM_SWEEP=200 timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py -q -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "variant and 188" > $O/case188_$v.log 2>&1; echo "$v rc=$?"; grep -o "worst normwise [0-9.e-]*\|1 passed\|1 failed\|\[[0-9.e-]*, [0-9.e-]*, [0-9.e-]*\]" $O/case188_$v.log | head -3
done
TMR_LIB_VARIANT=wsparse8 TMR_RANDOM_SWEEP=600 timeout -k 10 1000 python -u -m pytest tests/test_gpu_random.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/sweep600_wsparse8.log 2>&1; echo "sweep rc=$?"; tail -2 $O/sweep600_wsparse8.log
