# rocprofv3 sweep of both correlation kernels over the template side k, per regime:
# a kernel-trace run (durations) and one run per PMC counter pass (FETCH_SIZE, WRITE_SIZE,
# the SQ/GRBM group), each `kbench_xcorr.py --reps 3`.  Assembled by
# profiles/xcorr_sweep_assemble.py into profiles/xcorr_crossover.json + tmr_amd/xcorr_cost.json.
# Run from the repo root: gpurun -- bash profiles/gpu_xcorr_sweep.sh <label>
set -o pipefail
L=${1:-sweep}
OUT=gpurun_out/xsweep_$L
mkdir -p $OUT
export TMPDIR=/tmp
KS=1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31
regime() {  # regime <name> <kbench args...>
    local name=$1; shift
    local d=$OUT/$name
    mkdir -p $d
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d/trace -o t -- \
        python profiles/kbench_xcorr.py --reps 3 --ks $KS "$@" > $d/kbench.jsonl 2> $d/trace.err || return 1
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o p -- \
        python profiles/kbench_xcorr.py --reps 3 --ks $KS "$@" > $d/fetch.log 2>&1 || return 1
    timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o p -- \
        python profiles/kbench_xcorr.py --reps 3 --ks $KS "$@" > $d/write.log 2>&1 || return 1
    timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_LDS --output-format csv -d $d/core -o p -- \
        python profiles/kbench_xcorr.py --reps 3 --ks $KS "$@" > $d/core.log 2>&1 || return 1
    echo "regime $name done"
}
regime r128_e3_fp32 --images 64 --E 3 --H 128 --precision fp32 || exit 1
regime r192_e16_fp32 --images 8 --E 16 --H 192 --precision fp32 || exit 1
regime r128_e3_bf16 --images 64 --E 3 --H 128 --precision bf16 || exit 1
regime r192_e16_bf16 --images 8 --E 16 --H 192 --precision bf16 || exit 1
python profiles/xcorr_sweep_assemble.py $OUT $L > $OUT/assemble.log 2>&1 || { tail -5 $OUT/assemble.log; exit 1; }
cp profiles/xcorr_crossover.json $OUT/ && cp template-matching-and-regression-mapreduce_amd/xcorr_cost.json $OUT/
cat $OUT/assemble.log
