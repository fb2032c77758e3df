# xcorr experiment: GPU tests of the correlation kernels, then kbench_xcorr of
# the build variants (k = 3, the config-B mix 3..15, k = 15) and bench B.
# Run from the repo root: gpurun -- bash profiles/gpu_xcorr_exp.sh <variants...>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = main ] && v=""
  TMR_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "xcorr or golden or forward" --timeout 120 --timeout-method thread > gpurun_out/xcorr_tests.log 2>&1 || { echo "TESTS_FAILED ${v}"; tail -30 gpurun_out/xcorr_tests.log; exit 1; }
  echo "variant=${v:-main} $(tail -1 gpurun_out/xcorr_tests.log)"
done
for v in "$@"; do
  [ "$v" = main ] && v=""
  for kk in "--kmin 3 --kmax 3" "--kmin 3 --kmax 15" "--kmin 15 --kmax 15"; do
    TMR_LIB_VARIANT=$v timeout -k 10 120 python profiles/kbench_xcorr.py $kk --reps 7 > gpurun_out/kx.json 2>/dev/null || exit 1
    echo "variant=${v:-main} $(cat gpurun_out/kx.json)"
  done
  TMR_LIB_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/kb.json 2>/dev/null || exit 1
  echo "variant=${v:-main} bench B $(python -c 'import json;d=json.load(open("gpurun_out/kb.json"));print(d["value"],d["ms_per_step"])')"
done | tee gpurun_out/xcorr_exp.txt
