# Round 5 experiment: template_split + correlation interleaved per chunk of
# images (TMR_XCORR_CHUNK_IMAGES), so the A fragments are read back soon
# after they are written.  Parity with chunks of 2 images, then alternating
# bench runs at configs B and E.
# Run from the repo root: gpurun -- bash profiles/gpu_r05ah.sh
set -o pipefail
O=gpurun_out/r05ah
mkdir -p $O
export TMPDIR=/tmp
TMR_XCORR_CHUNK_IMAGES=2 timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "xcorr or headline or engine or precision" --timeout 200 --timeout-method thread > $O/tests_chunk2.log 2>&1
rc=$?; tail -1 $O/tests_chunk2.log
[ $rc -eq 0 ] || { echo TESTS_FAILED; grep -E "^FAILED" $O/tests_chunk2.log | head; exit 1; }
for rep in 1 2; do
  for ch in 0 4 8 16; do
    TMR_XCORR_CHUNK_IMAGES=$ch timeout -k 10 200 python bench.py --config B --steps 10 --warmup 2 --no-cpu-baseline --no-xcorr-classes > $O/B_c${ch}_$rep.json 2> $O/B_c${ch}_$rep.err || exit 1
    python -c "import json;d=json.load(open('$O/B_c${ch}_$rep.json'));x=d['roofline_xcorr'];print('B chunk $ch rep $rep',d['value'],x['avg_launch_ms'],x.get('hbm_frac'))"
  done
  for ch in 0 2 4; do
    TMR_XCORR_CHUNK_IMAGES=$ch timeout -k 10 200 python bench.py --config E --steps 4 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/E_c${ch}_$rep.json 2> $O/E_c${ch}_$rep.err || exit 1
    python -c "import json;d=json.load(open('$O/E_c${ch}_$rep.json'));x=d['roofline_xcorr'];print('E chunk $ch rep $rep',d['value'],x['avg_launch_ms'],x.get('hbm_frac'))"
  done
done
