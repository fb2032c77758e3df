# Round 4: host-side profile of the config-A module path (cProfile over the
# bench step loop) to see where the per-exemplar host turnaround goes.
set -o pipefail
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
timeout -k 10 300 python -m cProfile -o gpurun_out/r04f/module.prof bench.py --config A --path module --steps 60 --warmup 3 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || { tail -5 gpurun_out/r04f/bench.err; exit 1; }
python -c "
import pstats
p=pstats.Stats('gpurun_out/r04f/module.prof'); p.sort_stats('cumulative').print_stats(45)" > gpurun_out/r04f/module_cum.txt
python -c "
import pstats
p=pstats.Stats('gpurun_out/r04f/module.prof'); p.sort_stats('tottime').print_stats(40)" > gpurun_out/r04f/module_tot.txt
timeout -k 10 300 python -m cProfile -o gpurun_out/r04f/detect.prof bench.py --config A --steps 60 --warmup 3 --no-cpu-baseline --no-xcorr-classes > gpurun_out/r04f/bench_d.json 2> gpurun_out/r04f/bench_d.err || exit 1
python -c "
import pstats
p=pstats.Stats('gpurun_out/r04f/detect.prof'); p.sort_stats('tottime').print_stats(40)" > gpurun_out/r04f/detect_tot.txt
head -c 300 gpurun_out/r04f/bench.json
