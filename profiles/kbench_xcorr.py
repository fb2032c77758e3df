"""Micro-benchmark of the correlation kernel (tmr_xcorr) per template
size and kernel: for each k, B images x E exemplars of k x k templates on
fp [B,512,H,H]; HIP events around the correlation kernel's launch on its stream
(median of R repetitions; since round 6 the MFMA kernel's tmr_template_split
pass is outside the events -- earlier rounds' kbench figures include it).  One JSON line per (algo, k) with the SURVEY.md 8d roofline
figures: algorithmic bytes = read + write C*H*W fp32 per unit (fp read once
per unit, f_TM written), FLOPs = 2*C*(H-k+1)^2*k^2 per unit; HBM peak 8 TB/s,
fp32 VALU peak 157.3 TF.  --mixed runs the config-B mix (k uniform 3..15).

    python profiles/kbench_xcorr.py [--images 64] [--E 3] [--H 128] [--algos valu,mfma]
                                    [--ks 1,3,5,...] [--mixed] [--precision fp32|bf16|f16]
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


def run(eng, fp, ui, boxes, reps, heat=None):
    eng.match(fp, ui, boxes)  # warm
    eng.xcorr_events = []
    for _ in range(reps):
        if heat is not None:  # a decoder-sized MFMA launch right before (no sync)
            heat()
        eng.match(fp, ui, boxes)
    torch.cuda.synchronize()
    ms = float(np.median([s.elapsed_time(e) for s, e in eng.xcorr_events]))
    eng.xcorr_events = None
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--E", type=int, default=3)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--algos", default="valu,mfma")
    ap.add_argument("--ks", default="1,3,5,7,9,11,13,15,17,21,25,31")
    ap.add_argument("--mixed", action="store_true", help="config-B mix: k uniform over 3..15")
    ap.add_argument("--kmin", type=int, default=3)
    ap.add_argument("--kmax", type=int, default=15)
    ap.add_argument("--precision", default="fp32", help="MFMA operand precision: fp32 (3-term), bf16, f16")
    ap.add_argument("--heat-units", type=int, default=0,
                    help="before every timed launch, queue a 3-term decoder conv over this many units "
                         "(the chip's power state inside a bench step: the correlation follows the decoder)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, C, H = a.images, 512, a.H
    P = {k: v.to(dev) for k, v in synth.reference_state_dict(0).items()}
    eng = tmr.TMREngine(P, tmr.PathConfig(precision=a.precision))
    g = torch.Generator(device=dev).manual_seed(0)
    fp = torch.randn((B, C, H, H), device=dev, generator=g)
    ui = np.repeat(np.arange(B), a.E)
    sets = []
    if a.mixed:
        ex, ks = synth.exemplar_set(1, B, a.E, H, H, a.kmin, a.kmax)
        sets.append((f"{a.kmin}..{a.kmax}", ex.reshape(-1, 4), np.asarray(ks).reshape(-1)))
    else:
        for k in [int(x) for x in a.ks.split(",")]:
            ex, ks = synth.exemplar_set(1, B, a.E, H, H, k, k)
            sets.append((str(k), ex.reshape(-1, 4), np.asarray(ks).reshape(-1)))
    heat = None
    if a.heat_units:
        from tmr_amd._lib import PREC_CODES, call, ptr, stream
        from tmr_amd.engine import absmax, pack_split_w, pack_split_x
        hw_ = torch.randn((2048, 512, 3, 3), device=dev, generator=g) * 0.01
        hx = torch.randn((a.heat_units, 512, H, H), device=dev, generator=g)
        hwp, hwmax = pack_split_w(hw_, 512, "fp32")
        hxmax = absmax(hx)
        hxp = pack_split_x(hx, 3, "fp32", hxmax)
        del hx
        hb = torch.zeros(2048, device=dev)
        hout = torch.empty((a.heat_units, 2048, H, H), device=dev)

        def heat():
            call("tmr_split_conv", ptr(hxp), 512, None, None, 0, a.heat_units, H, H, 3,
                 PREC_CODES["fp32"], ptr(hwp), ptr(hwmax), ptr(hxmax), ptr(hb), 2048, 1, None, None, ptr(hout), 0,
                 stream())
    for name, boxes, ks in sets:
        flops = float(sum(2.0 * C * (H - k + 1) ** 2 * k * k for k in ks))
        nbytes = 2.0 * 4 * C * H * H * len(ks)
        for algo in a.algos.split(","):
            eng.xcorr_algo = algo
            try:
                ms = run(eng, fp, ui, boxes, a.reps, heat)
            except tmr.TMRError as e:
                print(json.dumps({"algo": algo, "k": name, "error": str(e)}), flush=True)
                continue
            print(json.dumps({"algo": algo, "prec": a.precision, "heat_units": a.heat_units, "k": name, "images": B, "E": a.E, "H": H, "ms": round(ms, 4),
                              "hbm_gbps": round(nbytes / ms / 1e6, 1),
                              "hbm_frac": round(nbytes / ms / 1e6 / 8000.0, 4),
                              "tflops": round(flops / ms / 1e9, 2),
                              "valu_frac": round(flops / ms / 1e9 / 157.3, 4)}), flush=True)


if __name__ == "__main__":
    main()
