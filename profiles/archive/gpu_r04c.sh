# Round 4: HIP-graph detect path + absmax fix: full -m gpu suite, smoke,
# config A with/without graphs (+ rocprof), the l2dma heads variant vs base, bench B.
set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "graph_replay" --timeout 120 --timeout-method thread > gpurun_out/r04c/graph_test.log 2>&1 || { echo GRAPH_TEST_FAILED; tail -25 gpurun_out/r04c/graph_test.log; exit 1; }
tail -1 gpurun_out/r04c/graph_test.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04c/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04c/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c/smoke.log 2>&1 || { tail -20 gpurun_out/r04c/smoke.log; exit 1; }
head -1 gpurun_out/r04c/smoke.log
for v in graph nograph; do
  if [ $v = graph ]; then X=""; else X="--no-graphs"; fi
  timeout -k 10 300 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline $X > gpurun_out/r04c/bench_A_$v.json 2> gpurun_out/r04c/bench_A_$v.err || { tail -5 gpurun_out/r04c/bench_A_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04c/bench_A_$v.json'));print('A $v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['config']['hip_graph'])"
done
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r04c/bench_A_module.json 2> gpurun_out/r04c/bench_A_module.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04c/bench_A_module.json'));print('A module',d['value'],d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04c/prof_A -o run -- python bench.py --config A --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04c/prof_A.log 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma --images 8 --E 16 --H 192 --kmax 31 > gpurun_out/r04c/kb_E_fp32.jsonl 2>&1 || exit 1
timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma,valu > gpurun_out/r04c/kb_B_fp32.jsonl 2>&1 || exit 1
grep -h '"ms"' gpurun_out/r04c/kb_*.jsonl
for v in base l2dma; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04c/var_$v.json 2> gpurun_out/r04c/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/r04c/var_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04c/var_$v.json'));print('$v heads ms',d['roofline']['avg_launch_ms'],'step',d['ms_per_step'])"
done
timeout -k 10 300 python bench.py > gpurun_out/r04c/bench_B.json 2> gpurun_out/r04c/bench_B.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04c/bench_B.json'));print('B',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['cpu_baseline']['value'])"
