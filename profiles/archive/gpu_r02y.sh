# r02y: template_split with the template staged in LDS per wave (old = previous build)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcorr" > gpurun_out/r02y_tests.log 2>&1 || { tail -30 gpurun_out/r02y_tests.log; exit 1; }
tail -1 gpurun_out/r02y_tests.log
for v in old new; do
  if [ $v = old ]; then export TMR_LIB_VARIANT=old; else unset TMR_LIB_VARIANT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02y_$v -o run -- python profiles/kbench_xcorr.py --algos mfma --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 --reps 3 > gpurun_out/r02y_$v.log 2>&1 || exit 1
done
unset TMR_LIB_VARIANT
python - <<'PY'
import sqlite3, collections
for v in ("old", "new"):
    c = sqlite3.connect(f"gpurun_out/prof_r02y_{v}/run_results.db")
    d = collections.defaultdict(list)
    for n, s, e in c.execute("select name,start,end from kernels"):
        if "template_split" in n or "xcorr_mfma" in n:
            d[n[:40]].append((e - s) / 1e6)
    print(v, {k: round(sum(x) / len(x), 3) for k, x in d.items()})
PY
