# r03pmc2: where the MFMA correlation's non-MFMA time goes at config E -- one rocprofv3
# --pmc pass of the issue/wait breakdown (SQ_WAIT_ANY = parked in s_waitcnt/barrier,
# SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_* = issuing) over bench.py --config E.
# Run from the repo root: gpurun -- bash profiles/gpu_r03pmc2.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc2_E -o p -- python bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline --no-xcorr-classes > gpurun_out/pmc2_E.log 2>&1 || { tail -20 gpurun_out/pmc2_E.log; exit 1; }
python profiles/pmc_csv.py 'xcorr_(rows|mfma)_kernel' gpurun_out/pmc2_E > gpurun_out/pmc2_E_xcorr.json 2>&1 || { cat gpurun_out/pmc2_E_xcorr.json | tail; exit 1; }
cat gpurun_out/pmc2_E_xcorr.json
python profiles/pmc_csv.py 'split_conv_kernel<\d+, \d+, 1>' gpurun_out/pmc2_E > gpurun_out/pmc2_E_heads.json 2>&1 || true
cat gpurun_out/pmc2_E_heads.json
