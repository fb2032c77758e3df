# Round 4: sparse-hi weight split (WH_BITS) -- precision and heads time, A/B in one call
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
for v in base wsparse8 wsparse6; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 200 python profiles/split_error.py >> $O/err.jsonl 2>> $O/err.err || exit 1
done
cat $O/err.jsonl
for rep in 1 2; do
for v in base wsparse8 wsparse6; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-xcorr-classes > $O/b_$v$rep.json 2> $O/b_$v$rep.err || exit 1
  python -c "import json;d=json.load(open('$O/b_$v$rep.json'));print('$v$rep',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
done
TMR_LIB_VARIANT=wsparse8 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread > $O/tests_wsparse8.log 2>&1; tail -3 $O/tests_wsparse8.log
