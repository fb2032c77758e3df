# Round 4: operand bit-density sweep of the one-term f16 decoder kernel
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python profiles/kbench_power.py --bits 11,9,8,7,6,4,2,1 > $O/bits.jsonl 2> $O/bits.err || { tail -5 $O/bits.err; exit 1; }
cat $O/bits.jsonl
