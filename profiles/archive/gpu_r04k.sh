# Round 4: sparse-hi template split in the MFMA correlation (TH_BITS) -- precision
# and correlation launch time, A/B in one call; then the full -m gpu suite on the
# committed tree (WH_BITS = 6 decoder weights).
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
for v in base tsparse8 tsparse6; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 200 python profiles/xcorr_error.py >> $O/err.jsonl 2>> $O/err.err || exit 1
done
cat $O/err.jsonl
for rep in 1 2; do
for v in base tsparse8 tsparse6; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 --algos mfma > $O/kb_E_$v$rep.jsonl 2>> $O/kb.err || exit 1
  TMR_LIB_VARIANT=$VAR timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --mixed --algos mfma > $O/kb_B_$v$rep.jsonl 2>> $O/kb.err || exit 1
  echo "$v$rep E $(cat $O/kb_E_$v$rep.jsonl) B $(cat $O/kb_B_$v$rep.jsonl)" | python -c "import sys,re;t=sys.stdin.read();print(t.split()[0], re.findall(r'\"ms\": ([0-9.]+)', t))"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -3 $O/gpu_tests.log
