# Round 4: the vectorised host prep (full -m gpu suite, bench B / A), and the
# decoder kernel's speed against its operand data (profiles/kbench_power.py).
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python profiles/kbench_power.py > $O/power.jsonl 2> $O/power.err || { tail -5 $O/power.err; exit 1; }
cat $O/power.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_B.json 2> $O/bench_B.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline > $O/bench_A.json 2> $O/bench_A.err || exit 1
for f in B A; do python -c "
import json;d=json.load(open('$O/bench_$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_B -o run -- python bench.py --steps 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_B.log 2>&1 || exit 1
