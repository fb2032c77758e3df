# Round 5, call p: config A (one image, 3 exemplars) -- where did the module
# path's +0.2 ms and detect's +0.1 ms (vs round 4) go?  Kernel traces of
# the detect and module paths, the module path's host phases, and the same
# two bench lines of the round-4 tree (ab/r04) on this box.
# Run from the repo root: gpurun -- bash profiles/gpu_r05p.sh
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
for t in cur r04; do
  d=.; [ $t != cur ] && d=ab/$t
  (cd $d && timeout -k 10 200 python bench.py --config A --steps 50 --warmup 3 --no-cpu-baseline) > $O/A_detect_$t.json 2> $O/A_detect_$t.err || { tail -5 $O/A_detect_$t.err; exit 1; }
  (cd $d && timeout -k 10 200 python bench.py --config A --path module --steps 30 --warmup 3 --no-cpu-baseline) > $O/A_module_$t.json 2> $O/A_module_$t.err || { tail -5 $O/A_module_$t.err; exit 1; }
  for f in A_detect_$t A_module_$t; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_Ad -o run -- python bench.py --config A --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_Ad.log 2>&1 || exit 1
python profiles/rocpd_summary.py $O/prof_Ad --label prof_Ad > $O/prof_Ad_kernel_stats.md 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_Am -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes > $O/prof_Am.log 2>&1 || exit 1
python profiles/rocpd_summary.py $O/prof_Am --label prof_Am > $O/prof_Am_kernel_stats.md 2>&1
(cd ab/r04 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ../../$O/prof_Am_r04 -o run -- python bench.py --config A --path module --steps 20 --warmup 3 --no-cpu-baseline --no-xcorr-classes) > $O/prof_Am_r04.log 2>&1 || exit 1
python profiles/rocpd_summary.py $O/prof_Am_r04 --label prof_Am_r04 > $O/prof_Am_r04_kernel_stats.md 2>&1
timeout -k 10 200 python profiles/module_phases.py --steps 40 > $O/phases.json 2> $O/phases.err || { tail -5 $O/phases.err; exit 1; }
tail -5 $O/phases.json
echo done
