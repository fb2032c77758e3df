# Round 5, call y: the correlation's A fragments built once per workgroup in
# LDS (TL 2, TMR_XCORR_AFRAG=lds when a unit's fragments fit 32 KB) vs the
# pre-expanded HBM fragments (split), config B, two reps; GPU correlation
# tests (bit-identity of the fragment sources) first.
# Run from the repo root: gpurun -- bash profiles/gpu_r05y.sh
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "xcorr or headline" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log
[ $rc -eq 0 ] || { echo TESTS_FAILED; grep -E "^FAILED|Error" $O/tests.log | head; exit 1; }
b() {  # b <tag> <afrag> <config>
  TMR_XCORR_AFRAG=$2 timeout -k 10 170 python bench.py --config $3 --no-cpu-baseline --no-xcorr-classes > $O/$1.json 2> $O/$1.err || { echo "BENCH_FAILED $1"; tail -5 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));x=d['roofline_xcorr'];print('$1',d['value'],d['ms_per_step'],x['algo'],x['avg_launch_ms'])"
}
for rep in 1 2; do b B_split_$rep split B && b B_lds_$rep lds B || exit 1; done
echo done
