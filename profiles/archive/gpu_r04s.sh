# Round 4: the fp-half store on a side stream (overlaps the f_TM record pack) -- GPU suite, A/B, rocprof B
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
for v in 1 0; do
timeout -k 10 300 python profiles/bench_variant.py overlap_store=$v -- --steps 10 --warmup 2 --no-cpu-baseline --no-xcorr-classes > $O/b_ov$v$r.json 2> $O/b_ov$v$r.err || exit 1
python -c "import json;d=json.load(open('$O/b_ov$v$r.json'));print('overlap=$v rep $r',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
done
for c in C E; do
for v in 1 0; do
timeout -k 10 300 python profiles/bench_variant.py overlap_store=$v -- --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-xcorr-classes > $O/b_${c}_ov$v.json 2> $O/b_${c}_ov$v.err || exit 1
python -c "import json;d=json.load(open('$O/b_${c}_ov$v.json'));print('$c overlap=$v',d['value'],d['ms_per_step'])"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_B -o run -- python bench.py --steps 3 --no-cpu-baseline > $O/prof_B.log 2>&1 || exit 1
