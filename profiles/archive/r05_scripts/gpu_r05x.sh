# Round 5, call x: the correlation's A-fragment ring (copy-free prefetch
# slots, XCORR_RING) vs the round-4 loop (xring0), and the ring's slot count
# (xpf3_N at config B, xpfwN at config E), one box; correlation launch ms
# from bench.py's HIP events.  GPU correlation tests on the new kernel first.
# Run from the repo root: gpurun -- bash profiles/gpu_r05x.sh
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "xcorr or headline or precision or template" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAILED; grep -E "^FAILED|Error" $O/tests.log | head; exit 1; }
b() {  # b <tag> <variant> <config>
  local tag=$1 v=$2 c=$3
  if [ $v = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$v; fi
  timeout -k 10 170 python bench.py --config $c --no-cpu-baseline --no-xcorr-classes > $O/$tag.json 2> $O/$tag.err || { echo "BENCH_FAILED $tag"; tail -5 $O/$tag.err; return 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));x=d['roofline_xcorr'];print('$tag',d['value'],d['ms_per_step'],x['algo'],x['avg_launch_ms'])"
}
for rep in 1 2; do
  b B_base_$rep base B && b B_xring0_$rep xring0 B && b E_base_$rep base E && b E_xring0_$rep xring0 E || exit 1
done
b B_xpf3_1 xpf3_1 B && b B_xpf3_3 xpf3_3 B && b E_xpfw2 xpfw2 E && b E_xpfw4 xpfw4 E && b C_base base C && b C_xring0 xring0 C || exit 1
echo done
