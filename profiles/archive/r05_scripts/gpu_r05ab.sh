# Round 5 final, part 1: PMC counters re-collected on the final kernels
# (profiles/gpu_pmc.sh), then a same-box A/B of the round-4 final tree (ab/r04)
# and this tree at configs B and E, alternating, two reps.
# Run from the repo root: gpurun -- bash profiles/gpu_r05ab.sh
set -o pipefail
bash profiles/gpu_pmc.sh r05 || { echo PMC_FAILED; exit 1; }
O=gpurun_out/r05ab
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for t in r04 cur; do
    d=.; [ $t != cur ] && d=ab/$t
    for c in B E; do
      (cd $d && timeout -k 10 240 python bench.py --config $c --no-cpu-baseline --no-xcorr-classes) > $O/ab_${t}_${c}_${rep}.json 2> $O/ab_${t}_${c}_${rep}.err || { echo "AB_FAILED $t $c"; tail -20 $O/ab_${t}_${c}_${rep}.err; exit 1; }
      python -c "import json;d=json.load(open('$O/ab_${t}_${c}_${rep}.json'));print('$t $c $rep',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
    done
  done
done
echo done
