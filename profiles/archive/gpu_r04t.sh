# Round 4: is the in-bench config-E correlation (~15 ms) slower than the kernel bench (~12 ms)
# because of the chip's power state after the decoder?  Same launch, with and without a
# decoder-sized MFMA launch queued right before each timed correlation.
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
for h in 0 24 0 24; do
timeout -k 10 300 python profiles/kbench_xcorr.py --images 8 --E 16 --H 192 --mixed --kmin 3 --kmax 31 --algos mfma --reps 5 --heat-units $h >> $O/kb_E.jsonl 2>> $O/kb.err || exit 1
done
cat $O/kb_E.jsonl
