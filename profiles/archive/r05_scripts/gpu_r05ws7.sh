# Round 5: the decoder weights' hi part at 7 significant bits (heads_variants
# wsparse7; 8 committed): config B speed (two reps, alternating with the
# committed build) and its worst errors over the 1200 + 1200-seed sweep.
# Run from the repo root: gpurun -- bash profiles/gpu_r05ws7.sh
set -o pipefail
O=gpurun_out/r05ws7
mkdir -p $O
export TMPDIR=/tmp
b() {  # b <tag> <variant>
  if [ $2 = base ]; then unset TMR_LIB_VARIANT; else export TMR_LIB_VARIANT=$2; fi
  timeout -k 10 200 python bench.py --config B --no-cpu-baseline --no-xcorr-classes > $O/$1.json 2> $O/$1.err || { echo "BENCH_FAILED $1"; tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
}
for rep in 1 2; do b B_base_$rep base && b B_ws7_$rep wsparse7 || exit 1; done
TMR_LIB_VARIANT=wsparse7 TMR_RANDOM_SWEEP=1200 timeout -k 10 500 python -u -m pytest tests/test_gpu_random.py -m gpu -q -s --timeout 450 --timeout-method thread > $O/random_sweep_ws7.log 2>&1
echo "sweep rc=$?"; tail -1 $O/random_sweep_ws7.log
