mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06e/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06e/tests.log
[ $rc -eq 0 ] || { grep -n "Error\|FAILED\|assert" gpurun_out/r06e/tests.log | head -20; exit 1; }
for c in B C E D; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/r06e/bench_$c.json 2> gpurun_out/r06e/bench_$c.err || exit 1; done
for c in B C E D; do python -c "import json;d=json.load(open('gpurun_out/r06e/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline_xcorr']['avg_launch_ms'],d['roofline_xcorr']['hbm_frac'],d['roofline_xcorr']['algo'])"; done
