# Round 4: module path (config A) host phases after the dummy-row fix, + cProfile of the steady state
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python profiles/module_phases.py --steps 100 > $O/phases.json 2> $O/phases.err || { tail $O/phases.err; exit 1; }
python -c "import json;d=json.load(open('$O/phases.json'));print(d['ms_per_image']);[print(k,v['mean_us']) for k,v in d['intervals'].items()]"
timeout -k 10 200 python profiles/module_phases.py --steps 100 --cprofile $O/cprof.txt > $O/phases_prof.json 2>> $O/phases.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_module100.json 2> $O/bench_A_module.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_A_module30.json 2>> $O/bench_A_module.err || exit 1
python -c "import json;[print(n,json.load(open('$O/bench_A_module%s.json'%n))['ms_per_step']) for n in ('100','30')]"
