# Round 4: the pruned tree (Winograd / fp32-MFMA decoders retired, macros ->
# constants) + grouped correlation launches: full -m gpu suite, smoke, the
# class-split sweep of the correlation (kbench_xcorr --splits), bench B and E.
set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04b/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04b/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04b/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04b/smoke.log 2>&1 || { tail -20 gpurun_out/r04b/smoke.log; exit 1; }
head -1 gpurun_out/r04b/smoke.log
fi
S_B='-;5;7;9;11;5,9;7,11;5,9,13'
S_E='-;9;11;13;17;9,17;11,19;7,13,19;9,15,21;7,11,15,19,23;5,9,13,17,21,25'
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma --splits="$S_B" > gpurun_out/r04b/split_B_fp32.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma --precision bf16 --splits="$S_B" > gpurun_out/r04b/split_B_bf16.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma --images 8 --E 16 --H 192 --kmax 31 --splits="$S_E" > gpurun_out/r04b/split_E_fp32.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma --images 8 --E 16 --H 192 --kmax 31 --precision bf16 --splits="$S_E" > gpurun_out/r04b/split_E_bf16.jsonl 2>&1 || exit 1
grep -h '"split"' gpurun_out/r04b/split_*.jsonl | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['prec'],d['H'],d['split'],d['ms'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04b/bench_B.json 2> gpurun_out/r04b/bench_B.err || exit 1
timeout -k 10 300 python bench.py --config E --no-cpu-baseline > gpurun_out/r04b/bench_E.json 2> gpurun_out/r04b/bench_E.err || exit 1
for c in B E; do python -c "import json;d=json.load(open('gpurun_out/r04b/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d['roofline_xcorr']['avg_launch_ms'])"; done
# heads-kernel timing-only variants (profiles/heads_variants.py; wrong results by design)
for v in base nobar nowait noacc0 noepi nodma; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04b/var_$v.json 2> gpurun_out/r04b/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/r04b/var_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04b/var_$v.json'));print('$v heads ms',d['roofline']['avg_launch_ms'],'step',d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --config A --no-cpu-baseline > gpurun_out/r04b/bench_A.json 2> gpurun_out/r04b/bench_A.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04b/prof_A -o run -- python bench.py --config A --steps 20 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04b/prof_A.log 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04b/bench_A.json'));print('A',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
