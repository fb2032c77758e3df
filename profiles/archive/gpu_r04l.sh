# Round 4: module path (config A) host phases; back-to-back graph replay test
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread -k "graph" > $O/graph_tests.log 2>&1; tail -2 $O/graph_tests.log
timeout -k 10 200 python profiles/module_phases.py --steps 100 > $O/phases.json 2> $O/phases.err || { tail $O/phases.err; exit 1; }
cat $O/phases.json
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_A_module.json 2> $O/bench_A_module.err || exit 1
python -c "import json;d=json.load(open('$O/bench_A_module.json'));print('module',d['ms_per_step'])"
