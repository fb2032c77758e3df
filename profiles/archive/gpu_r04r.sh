# Round 4: why the VALU correlation sits below the HBM roof at k <= 9 --
# PMC passes over (a) bench.py config B's k<=9 class launch (the by_class line) and
# (b) single-k kernel-bench launches at k = 3 and 9 (64 images x 3 units, 128^2).
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="WRITE_SIZE"
P3="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS"
P4="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/bench_p$i -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_p$i.log 2>&1 || exit 1
  for k in 3 9; do
    timeout -s KILL 100 rocprofv3 --pmc $P --output-format csv -d $O/k${k}_p$i -o p -- python profiles/kbench_xcorr.py --algos valu --ks $k --reps 2 > $O/k${k}_p$i.log 2>&1 || exit 1
  done
  echo "pass $i done"
done
timeout -s KILL 150 rocprofv3 --pmc $P4 --output-format csv -d $O/bench_p4 -o p -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_p4.log 2>&1 && echo "pass 4 done" || echo "pass 4 failed"
python profiles/pmc_csv.py xcorr_rows $O/bench_p1 $O/bench_p2 $O/bench_p3 > $O/bench_class.json && cat $O/bench_class.json
for k in 3 9; do python profiles/pmc_csv.py xcorr_rows $O/k${k}_p1 $O/k${k}_p2 $O/k${k}_p3 > $O/k$k.json && cat $O/k$k.json; done
python profiles/pmc_csv.py xcorr_rows $O/bench_p4 > $O/bench_p4.json 2>/dev/null && cat $O/bench_p4.json || true
