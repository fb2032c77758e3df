# r02x: bench lines for all configs + rocprofv3 kernel-trace of B and E (after the r02 kernel changes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02x_bench_B.json 2> gpurun_out/r02x_bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02x_bench_C.json 2> gpurun_out/r02x_bench_C.err || exit 1
timeout -k 10 300 python bench.py --config D --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02x_bench_D.json 2> gpurun_out/r02x_bench_D.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02x_bench_E.json 2> gpurun_out/r02x_bench_E.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02x_bench_A_module.json 2> gpurun_out/r02x_bench_A_module.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02x_bench_A_detect.json 2> gpurun_out/r02x_bench_A_detect.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02x_B -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02x_B.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02x_E -o run -- python bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02x_E.log 2>&1 || exit 1
python - <<'PY'
import json
for c in ["B","C","D","E","A_module","A_detect"]:
    d=json.loads(open(f"gpurun_out/r02x_bench_{c}.json").read().strip().splitlines()[-1])
    print(c, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["executed_frac"], d["roofline_xcorr"]["algo"], d["roofline_xcorr"]["avg_launch_ms"], d.get("cpu_baseline"))
PY
