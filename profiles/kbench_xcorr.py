"""Micro-benchmark of the correlation step at the config-B shape: 64 images x
3 exemplars, fp [64,512,128,128], templates 3..15 (TMREngine.match =
tmr_templates + tmr_xcorr with the fused max |f_TM|).  HIP events on the
launch stream, median of R repetitions; prints one JSON line with the VALU
roofline fraction (2*C*(H-h+1)(W-w+1)*h*w flops per unit, 157.3 TF fp32).

    python profiles/kbench_xcorr.py [--images 64] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

tmr = load_package()
from tmr_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--E", type=int, default=3)
    ap.add_argument("--kmax", type=int, default=15)
    ap.add_argument("--kmin", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, C, H = a.images, 512, 128
    P = {k: v.to(dev) for k, v in synth.reference_state_dict(0).items()}
    eng = tmr.TMREngine(P, tmr.PathConfig())
    g = torch.Generator(device=dev).manual_seed(0)
    fp = torch.randn((B, C, H, H), device=dev, generator=g)
    ex, ks = synth.exemplar_set(1, B, a.E, H, H, a.kmin, a.kmax)
    ui = np.repeat(np.arange(B), a.E)
    boxes = ex.reshape(-1, 4)
    flops = 0.0
    for k in np.asarray(ks).reshape(-1):
        k = int(k)
        flops += 2.0 * C * (H - k + 1) ** 2 * k * k
    eng.match(fp, ui, boxes)
    ts = []
    for _ in range(a.reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        eng.match(fp, ui, boxes)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ms = float(np.median(ts))
    out_bytes = B * a.E * C * H * H * 4
    print(json.dumps({"images": B, "E": a.E, "k": [a.kmin, a.kmax], "ms": round(ms, 3), "gflop": round(flops / 1e9, 1),
                      "tflops": round(flops / ms / 1e9, 1), "frac_valu": round(flops / ms / 1e9 / 157.3, 3),
                      "hbm_gbps_out": round(out_bytes / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
