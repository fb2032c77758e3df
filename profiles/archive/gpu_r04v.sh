# Round 4: cProfile of the module path's steady state (config A) after the host-time cuts
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python profiles/module_phases.py --steps 200 --cprofile $O/cprof.txt > $O/phases.json 2> $O/phases.err || { tail $O/phases.err; exit 1; }
head -60 $O/cprof.txt
