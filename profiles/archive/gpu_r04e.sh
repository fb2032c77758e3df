# Round 4: correlation A/B in one call -- the MFMA kernel's term-major order
# (libtmr.so) vs the previous order (libtmr_xold.so, xcorr.hip of e4094b4), and
# the VALU kernel, on the config-B and config-E mixes; config A module path
# with graphs.
set -o pipefail
mkdir -p gpurun_out/r04e
export TMPDIR=/tmp
for rep in 1 2; do
for v in new xold; do
  if [ $v = new ]; then VAR=""; else VAR=xold; fi
  TMR_LIB_VARIANT=$VAR timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma,valu > gpurun_out/r04e/kb_B_$v$rep.jsonl 2>&1 || exit 1
  TMR_LIB_VARIANT=$VAR timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma,valu --images 8 --E 16 --H 192 --kmax 31 > gpurun_out/r04e/kb_E_$v$rep.jsonl 2>&1 || exit 1
  TMR_LIB_VARIANT=$VAR timeout -k 10 300 python profiles/kbench_xcorr.py --mixed --algos mfma --precision bf16 > gpurun_out/r04e/kb_C_$v$rep.jsonl 2>&1 || exit 1
  grep -h '"ms"' gpurun_out/r04e/kb_*_$v$rep.jsonl | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v$rep',d['algo'],d['prec'],d['H'],d['ms'])"
done
done
timeout -k 10 300 python bench.py --config A --path module --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/r04e/bench_A_module.json 2> gpurun_out/r04e/bench_A_module.err || { tail -5 gpurun_out/r04e/bench_A_module.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04e/bench_A_module.json'));print('A module',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['config']['hip_graph'])"
timeout -k 10 300 python bench.py --config A --path module --steps 50 --warmup 3 --no-cpu-baseline --no-graphs > gpurun_out/r04e/bench_A_module_nograph.json 2> gpurun_out/r04e/bench_A_module_nograph.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r04e/bench_A_module_nograph.json'));print('A module nograph',d['value'],d['ms_per_step'])"
