# Round 4: what the correlation waits on -- timing variants (wrong results by construction):
# band staging from L2 (xl2band), A fragments from L1/L2 (xl2a); config-B and config-E mixes
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for v in base xl2band xl2a; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 200 python profiles/kbench_xcorr.py --images 64 --E 3 --H 128 --mixed --algos mfma > $O/kb_B_$v$rep.jsonl 2>> $O/kb.err || exit 1
  TMR_LIB_VARIANT=$VAR timeout -k 10 200 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 --algos mfma > $O/kb_E_$v$rep.jsonl 2>> $O/kb.err || exit 1
  echo "$v$rep B $(python -c "import json;print(json.loads(open('$O/kb_B_$v$rep.jsonl').readline())['ms'])") E $(python -c "import json;print(json.loads(open('$O/kb_E_$v$rep.jsonl').readline())['ms'])")"
done
done
