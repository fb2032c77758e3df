# Round 5: graph signatures with the parameter names' order cached (host time
# of the module path); the graph-replay GPU tests, then config A detect /
# module, two reps each.
# Run from the repo root: gpurun -- bash profiles/gpu_r05aa.sh
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "graph or module" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAILED; grep -E "^FAILED" $O/tests.log | head; exit 1; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline > $O/A_detect_$rep.json 2> $O/A_detect_$rep.err || exit 1
  timeout -k 10 200 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > $O/A_module_$rep.json 2> $O/A_module_$rep.err || exit 1
  for f in A_detect_$rep A_module_$rep; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
done
timeout -k 10 200 python profiles/module_phases.py --steps 40 > $O/phases.json 2> $O/phases.err || exit 1
python -c "import json;d=json.load(open('$O/phases.json'));print({k:v['mean_us'] for k,v in d['intervals'].items()})"
