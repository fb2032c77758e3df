# r02a: new headline / call-form tests first (verbose, per-test timeout), then
# the full -m gpu suite, smoke, one bench B line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/r02a_headline.log 2>&1 || { echo HEADLINE_FAILED; tail -30 gpurun_out/r02a_headline.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r02a_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02a_gpu_tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/r02a_smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r02a_bench_B.json 2> gpurun_out/r02a_bench_B.err || exit 1
tail -3 gpurun_out/r02a_headline.log; cat gpurun_out/r02a_smoke.log; cat gpurun_out/r02a_bench_B.json
timeout -k 10 300 python bench.py --config A --path module --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02a_bench_A_module.json 2> gpurun_out/r02a_bench_A_module.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02a_bench_A_detect.json 2> gpurun_out/r02a_bench_A_detect.err || exit 1
cat gpurun_out/r02a_bench_A_module.json gpurun_out/r02a_bench_A_detect.json
