# r02j: NMS reduce over 256 threads per image + chain over surviving rows (old vs new at config E), parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "nms" > gpurun_out/r02j_tests.log 2>&1 || exit 1
TMR_LIB_VARIANT=old timeout -k 10 300 python bench.py --config E --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02j_E_old.json 2> gpurun_out/r02j_E_old.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r02j_E_new.json 2> gpurun_out/r02j_E_new.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02j_E -o run -- python bench.py --config E --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02j_E.log 2>&1 || exit 1
tail -2 gpurun_out/r02j_tests.log
python - <<'PY'
import json
for v in ("old","new"):
    d=json.loads(open(f"gpurun_out/r02j_E_{v}.json").read().strip().splitlines()[-1])
    print(v, d["value"], d["ms_per_step"])
PY
