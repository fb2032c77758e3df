"""Diagnostic: is this host's torch.exp (CPU) the same function as the one the
reference-exp table was recorded from?  Prints the CPU model, torch/MKL info
and the mismatch counts of torch.exp vs (correctly rounded, table emulation)."""
import os, sys, platform
import numpy as np, torch
sys.path.insert(0, os.getcwd())
from tmr_import import load_package
load_package()
from tmr_amd import exp_table
try:
    cpu = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].strip()
except Exception:
    cpu = platform.processor()
print(cpu, torch.__version__, torch.backends.cpu.get_cpu_capability(), flush=True)
raw = exp_table.read()
rng = np.random.default_rng(7)
x = np.concatenate([rng.normal(0, 3, 30000), rng.normal(0, 1e-3, 10000), -np.abs(rng.normal(0, 1e-6, 10000))]).astype(np.float32)
t = torch.exp(torch.from_numpy(x)).numpy()
e = np.exp(x.astype(np.float64)); cr = e.astype(np.float32)
hit = exp_table.lookup_host(x, raw)
emu = np.where(hit, np.where(e > cr.astype(np.float64), np.nextafter(cr, np.float32(np.inf)), np.nextafter(cr, np.float32(-np.inf))), cr)
print("torch!=cr", int((t.view(np.uint32) != cr.view(np.uint32)).sum()), "torch!=table-emulation", int((t.view(np.uint32) != emu.view(np.uint32)).sum()), "of", x.size)
