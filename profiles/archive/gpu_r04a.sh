# Round 4 first GPU call: (1) a clean checkout (git archive of HEAD, shipped
# as clean_head.tar) builds and passes smoke() on the box with nothing from
# the working tree; (2) the full -m gpu suite incl. the RCCL world-1 tests;
# (3) bench B.  Run from the repo root: gpurun -- bash profiles/archive/gpu_r04a.sh
set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
CL=$TMPDIR/tmr_clean_$$
rm -rf $CL && mkdir -p $CL && tar -xf clean_head.tar -C $CL || exit 1
( cd $CL && ls template-matching-and-regression-mapreduce_amd > $OLDPWD/gpurun_out/r04a/clean_ls.txt && \
  timeout -k 10 400 python -c "import __graft_entry__ as g; g.build(); print('clean build ok')" > $OLDPWD/gpurun_out/r04a/clean_build.log 2>&1 && \
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OLDPWD/gpurun_out/r04a/clean_smoke.log 2>&1 ) || { echo CLEAN_FAILED; tail -20 gpurun_out/r04a/clean_*.log; exit 1; }
tail -2 gpurun_out/r04a/clean_build.log; tail -3 gpurun_out/r04a/clean_smoke.log
sha256sum $CL/template-matching-and-regression-mapreduce_amd/exp_ref.bin > gpurun_out/r04a/clean_exp_sha.txt
rm -rf $CL
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04a/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04a/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04a/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r04a/bench_B.json 2> gpurun_out/r04a/bench_B.err || exit 1
cat gpurun_out/r04a/bench_B.json
