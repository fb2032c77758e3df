# Round 4: module path host-time changes -- full GPU suite, module phases, bench A (detect, module)
set -o pipefail
O=gpurun_out/${1:-r04n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python profiles/module_phases.py --steps 100 > $O/phases.json 2> $O/phases.err || { tail $O/phases.err; exit 1; }
python -c "import json;d=json.load(open('$O/phases.json'));print(d['ms_per_image']);[print(k,v['mean_us']) for k,v in d['intervals'].items()]"
for r in 1 2; do
timeout -k 10 300 python bench.py --config A --path module --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_module$r.json 2> $O/bench_A_module.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_detect$r.json 2> $O/bench_A_detect.err || exit 1
python -c "import json;[print(n,json.load(open('$O/bench_A_%s$r.json'%n))['ms_per_step']) for n in ('module','detect')]"
done
