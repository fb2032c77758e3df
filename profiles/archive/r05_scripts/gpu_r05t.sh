# Round 5, call t: the heads launch's image-major order at config E (16 units
# per image) on / off (TMR_HEADS_IMAGE_MAJOR_MAX 255 / 8), two reps, one box.
# Run from the repo root: gpurun -- bash profiles/gpu_r05t.sh
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for m in 255 8; do
    TMR_HEADS_IMAGE_MAJOR_MAX=$m timeout -k 10 240 python bench.py --config E --no-cpu-baseline --no-xcorr-classes > $O/E_im${m}_$rep.json 2> $O/E_im${m}_$rep.err || { echo FAILED; tail -20 $O/E_im${m}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/E_im${m}_$rep.json'));print('E im$m $rep',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
  done
done
echo done
