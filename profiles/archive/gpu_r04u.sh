# Round 4: detect's in-forward small NMS -- parity/headline tests, config A benches, phases
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_abi_host.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python bench.py --config A --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_detect$r.json 2> $O/bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 100 --warmup 3 --no-cpu-baseline > $O/bench_A_module$r.json 2> $O/bench_A_module.err || exit 1
python -c "import json;[print(n,json.load(open('$O/bench_A_%s$r.json'%n))['ms_per_step']) for n in ('detect','module')]"
done
