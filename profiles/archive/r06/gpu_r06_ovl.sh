# Round 6 same-box A/B: the decoder's fp half on a side stream concurrent with the correlation
# (overlap_fp_half=1) vs in order (0), alternating, two reps; configs B and E.
L=${1:-r06ovlab}; O=gpurun_out/$L; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do for v in 1 0; do for c in B E; do
timeout -k 10 300 python profiles/bench_variant.py overlap_fp_half=$v -- --config $c --no-cpu-baseline > $O/${c}_ovl${v}_$rep.json 2> $O/${c}_ovl${v}_$rep.err || exit 1
done; done; done
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline_xcorr']['avg_launch_ms'])"; done
