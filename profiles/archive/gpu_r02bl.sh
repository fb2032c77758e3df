# r02bl: tiled upsample bit-exactness at edge sizes and the projection order test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "upsample2x_tiled or golden_forward or forward" > gpurun_out/r02bl_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02bl_tests.log; exit 1; }
tail -1 gpurun_out/r02bl_tests.log
