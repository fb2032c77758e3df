# r03final: round-3 final check of the final tree (labels r03f2): full -m gpu suite (incl. the config A/C/D
# graded-batch tests), the box's peaks (peakbench), smoke(), bench lines of every config (B with the default K/W and CPU
# baseline), rocprofv3 kernel traces of B, C and E, and the --gpus 2 launcher over gloo.
# PMC passes first (profiles/gpu_pmc.sh r03f2 -> profiles/pmc_by_config.json on the box, so the
# bench lines below carry this round's traffic).
# Run from the repo root: gpurun --timeout 1200 -- bash profiles/gpu_r03f2.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash profiles/gpu_pmc.sh r03f2 > gpurun_out/r03f2_pmc.log 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/r03f2_pmc.log; exit 1; }
tail -12 gpurun_out/r03f2_pmc.log
cp gpurun_out/pmc_r03f2/pmc_by_config.json profiles/pmc_by_config.json || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03f2_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03f2_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03f2_gpu_tests.log
grep -E "worst normwise map error|mean kept|config A kept" gpurun_out/r03f2_gpu_tests.log
timeout -k 10 120 ./profiles/peakbench/peakbench > gpurun_out/r03f2_peaks.json 2> gpurun_out/r03f2_peaks.err || { cat gpurun_out/r03f2_peaks.err; exit 1; }
cat gpurun_out/r03f2_peaks.json
python -c "import json;d=json.load(open('gpurun_out/r03f2_peaks.json'));d['source']='profiles/peakbench (round r03f2 box)';json.dump(d,open('profiles/peaks_measured.json','w'),indent=1)" || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03f2_smoke.log 2>&1 || { tail -20 gpurun_out/r03f2_smoke.log; exit 1; }
tail -1 gpurun_out/r03f2_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03f2_bench_B.json 2> gpurun_out/r03f2_bench_B.err || exit 1
timeout -k 10 300 python bench.py --config C > gpurun_out/r03f2_bench_C.json 2> gpurun_out/r03f2_bench_C.err || exit 1
timeout -k 10 300 python bench.py --config D --steps 10 --warmup 2 > gpurun_out/r03f2_bench_D.json 2> gpurun_out/r03f2_bench_D.err || exit 1
timeout -k 10 300 python bench.py --config E --steps 5 --warmup 2 > gpurun_out/r03f2_bench_E.json 2> gpurun_out/r03f2_bench_E.err || exit 1
timeout -k 10 300 python bench.py --config A --steps 30 --warmup 5 > gpurun_out/r03f2_bench_A_detect.json 2> gpurun_out/r03f2_bench_A_detect.err || exit 1
timeout -k 10 300 python bench.py --config A --path module --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r03f2_bench_A_module.json 2> gpurun_out/r03f2_bench_A_module.err || exit 1
for c in B C D E A_detect A_module; do python -c "import json;d=json.loads(open('gpurun_out/r03f2_bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];x=d['roofline_xcorr'];print('$c',d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['path_frac'],r['traffic'],x['algo'],x['avg_launch_ms'],x['dram_min_frac'],d['cpu_baseline'] and d['cpu_baseline']['value'])"; done
for c in B C E; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03f2_$c -o run -- python bench.py --config $c --steps 2 --no-cpu-baseline --no-xcorr-classes > gpurun_out/prof_r03f2_$c.log 2>&1 || exit 1
  python profiles/rocpd_summary.py gpurun_out/prof_r03f2_$c --label "prof_r03f2_$c: bench.py --config $c --steps 2" > gpurun_out/r03f2_bench_${c}_kernel_stats.md || exit 1
  tail -3 gpurun_out/r03f2_bench_${c}_kernel_stats.md
done
TMR_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-xcorr-classes > gpurun_out/r03f2_bench_B_gpus2_gloo.json 2> gpurun_out/r03f2_bench_B_gpus2_gloo.err || { tail -20 gpurun_out/r03f2_bench_B_gpus2_gloo.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/r03f2_bench_B_gpus2_gloo.json') if l.startswith('{')][-1]);print('gpus2 gloo rehearsal', d['n_gpus'], d['value'], d['config']['parallelism'])"
TMR_FULL_PARITY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -m gpu -k full_batch -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r03f2_full_parity.log 2>&1 || { echo FULL_PARITY_FAILED; tail -40 gpurun_out/r03f2_full_parity.log; exit 1; }
tail -1 gpurun_out/r03f2_full_parity.log
