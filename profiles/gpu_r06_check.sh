# Round 6 check of the working tree: the full -m gpu suite, then bench lines for
# configs B C D E and A (detect and module paths).
# Run from the repo root: gpurun -- bash profiles/gpu_r06_check.sh <label>
set -o pipefail
L=${1:-r06chk}
O=gpurun_out/$L
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -n "Error\|FAILED\|assert" $O/tests.log | head -20; exit 1; }
for c in B C E D; do timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; done
timeout -k 10 300 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline > $O/bench_A_detect.json 2> $O/bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_A_module.json 2> $O/bench_A_module.err || exit 1
for c in B C E D A_detect A_module; do python -c "import json;d=json.load(open('$O/bench_$c.json'));x=d['roofline_xcorr'];print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],x['avg_launch_ms'],x['hbm_frac'],x['algo'])"; done
