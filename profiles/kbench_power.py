"""Does the split decoder kernel's speed depend on its operand DATA?

The heads-launch variants (profiles/heads_variants.py) left
the MFMA issue at a power-limited clock as the bound, and the variant that fed
the MFMAs constant LDS contents ran 30% faster.  This times
tmr_split_conv (3-term fp32 contract, 3x3, 512 -> 2048 channels at
128^2, a batch of units) on the SAME launch with different activation data:
standard normal, LayerNorm'd SAM-like features upsampled x2 (smooth), a real
correlation output (f_TM), a constant, and zeros; weights reference-init or
zero.  HIP events around each launch on its stream, median of --reps.

    python profiles/kbench_power.py [--units 48] [--reps 5]
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
from tmr_amd._lib import PREC_CODES, call, load, ptr, stream  # noqa: E402
from tmr_amd.engine import absmax, pack_split_w, pack_split_x  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--units", type=int, default=48)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--bits", default="", help="instead: the one-term f16 kernel with weights (then "
                    "activations) rounded to these numbers of significant bits, e.g. 11,8,6,4,2")
    a = ap.parse_args()
    if a.bits:
        return bits_sweep(a)
    dev = torch.device("cuda:0")
    U, C, N, H, W, ks = a.units, 512, 2048, 128, 128, 3
    g = torch.Generator(device=dev).manual_seed(0)
    w = torch.randn((N, C, ks, ks), device=dev, generator=g) * 0.01
    b = torch.zeros(N, device=dev)
    P = {k: v.to(dev) for k, v in synth.reference_state_dict(0).items()}
    eng = tmr.TMREngine(P, tmr.PathConfig())
    feats = torch.from_numpy(synth.sam_features(3, max(1, U // 3), 256, 64, 64)).to(dev)
    fp, _ = eng.project(feats)
    ex, _ = synth.exemplar_set(4, fp.shape[0], 3, H, W, 3, 15)
    ui = np.repeat(np.arange(fp.shape[0]), 3)[:U]
    ftm, _ = eng.match(fp, ui, ex.reshape(-1, 4)[:U])
    data = {
        "normal": torch.randn((U, C, H, W), device=dev, generator=g),
        "sam_up2x": torch.nn.functional.interpolate(
            torch.from_numpy(synth.sam_features(5, U, C, 64, 64)).to(dev), scale_factor=2, mode="bilinear",
            align_corners=False),
        "f_tm": ftm.float().contiguous(),
        "fp_proj": fp.index_select(0, torch.from_numpy(ui).to(dev)).contiguous(),
        "const": torch.full((U, C, H, W), 0.37, device=dev),
        "zeros": torch.zeros((U, C, H, W), device=dev),
    }
    out = torch.empty((U, N, H, W), device=dev)
    pc = PREC_CODES[a.precision]
    for wname, ww in (("w_ref", w), ("w_zero", torch.zeros_like(w))):
        wp, wmax = pack_split_w(ww, C, a.precision)
        for name, x in data.items():
            xmax = absmax(x)
            xp = pack_split_x(x, ks, a.precision, xmax)
            ms = []
            for _ in range(a.reps + 1):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                call("tmr_split_conv", ptr(xp), C, None, None, 0, U, H, W, ks, pc, ptr(wp), ptr(wmax),
                     ptr(xmax), ptr(b), N, 1, None, None, ptr(out), 0, stream())
                e.record()
                torch.cuda.synchronize()
                ms.append(s.elapsed_time(e))
            del xp
            print(json.dumps({"weights": wname, "data": name, "precision": a.precision, "units": U,
                              "ms": round(float(np.median(ms[1:])), 3),
                              "x_absmax": round(float(x.abs().max()), 4)}), flush=True)


def round_bits(t: torch.Tensor, k: int) -> torch.Tensor:
    """t rounded to k significant bits (round to nearest even by the fp32 add trick)."""
    m, e = torch.frexp(t)
    scale = torch.ldexp(torch.ones_like(m), torch.full_like(e, k))
    return torch.ldexp(torch.round(m * scale) / scale, e)


def bits_sweep(a):
    """One fp16 MFMA term per product: does an operand with fewer significant
    bits (fewer partial products in the multiplier) make the launch faster?"""
    dev = torch.device("cuda:0")
    U, C, N, H, W, ks = a.units, 512, 2048, 128, 128, 3
    g = torch.Generator(device=dev).manual_seed(0)
    w0 = torch.randn((N, C, ks, ks), device=dev, generator=g) * 0.01
    x0 = torch.randn((U, C, H, W), device=dev, generator=g)
    b = torch.zeros(N, device=dev)
    out = torch.empty((U, N, H, W), device=dev)
    pc = PREC_CODES["f16"]
    for which in ("w", "x"):
        for k in [int(v) for v in a.bits.split(",")]:
            w = round_bits(w0, k) if which == "w" else w0
            x = round_bits(x0, k) if which == "x" else x0
            wp, wmax = pack_split_w(w, C, "f16")
            xmax = absmax(x)
            xp = pack_split_x(x, ks, "f16", xmax)
            ms = []
            for _ in range(a.reps + 1):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                call("tmr_split_conv", ptr(xp), C, None, None, 0, U, H, W, ks, pc, ptr(wp), ptr(wmax),
                     ptr(xmax), ptr(b), N, 1, None, None, ptr(out), 0, stream())
                e.record()
                torch.cuda.synchronize()
                ms.append(s.elapsed_time(e))
            print(json.dumps({"rounded": which, "bits": k, "precision": "f16", "units": U,
                              "ms": round(float(np.median(ms[1:])), 3)}), flush=True)


if __name__ == "__main__":
    main()
