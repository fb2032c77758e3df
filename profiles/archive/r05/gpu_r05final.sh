# Round 5 final tree: full -m gpu suite, smoke, every bench line (B with the
# CPU baseline; C, D, E; A detect / module), rocprofv3 kernel traces of B and
# E, and a 2-rank gloo rehearsal on the one card (physical_gpus = 1).
# Run from the repo root: gpurun -- bash profiles/gpu_r05final.sh [label]
set -o pipefail
O=gpurun_out/${1:-r05final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_B.json 2> $O/bench_B.err || exit 1
for c in C D E; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
timeout -k 10 300 python bench.py --config A --steps 50 --warmup 3 > $O/bench_A_detect.json 2> $O/bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_A_module.json 2> $O/bench_A_module.err || exit 1
for f in B C D E A_detect A_module; do python -c "
import json;d=json.load(open('$O/bench_$f.json'));r=d['roofline'];x=d['roofline_xcorr']
print('$f',d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['traffic'],x['avg_launch_ms'],x.get('hbm_frac'),(d.get('cpu_baseline') or {}).get('value'))"; done
for c in B E; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python bench.py --config $c --steps 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_$c.log 2>&1 || exit 1
  python profiles/rocpd_summary.py $O/prof_$c --label prof_$c > $O/prof_${c}_kernel_stats.md 2>&1
done
head -8 $O/prof_B_kernel_stats.md
TMR_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/bench_B_gpus2_gloo_1gpu.json 2> $O/bench_B_gpus2_gloo_1gpu.err || exit 1
grep -h '^{' $O/bench_B_gpus2_gloo_1gpu.json | python -c "import sys,json;d=json.loads(sys.stdin.read());print('gloo x2',d['n_gpus'],d['physical_gpus'],d['exchange'],d['value'])"
