# Round 4: module-path HIP graphs: the graph tests first, then the full -m gpu
# suite, config A detect / module, bench B.
set -o pipefail
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q -k "graph_replay" --timeout 120 --timeout-method thread > gpurun_out/r04d/graph_tests.log 2>&1 || { echo GRAPH_TESTS_FAILED; tail -30 gpurun_out/r04d/graph_tests.log; exit 1; }
tail -1 gpurun_out/r04d/graph_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04d/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r04d/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04d/gpu_tests.log
for p in detect module; do
  timeout -k 10 300 python bench.py --config A --path $p --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/r04d/bench_A_$p.json 2> gpurun_out/r04d/bench_A_$p.err || { tail -5 gpurun_out/r04d/bench_A_$p.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04d/bench_A_$p.json'));print('A $p',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['config']['hip_graph'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04d/prof_A_module -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04d/prof_A_module.log 2>&1 || exit 1
