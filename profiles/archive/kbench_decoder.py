"""Micro-benchmark of the decoder kernels at the config-B shape (128x128 maps,
N = 2048 output channels, K = 512 input channels for the per-unit f_TM half):
tmr_wino_conv_heads / tmr_conv_heads (and the *_store fp-half variants), HIP
events on the launch stream, median of R repetitions.  Prints one JSON line.

    python profiles/kbench_decoder.py [--units 48] [--reps 5]
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
from tmr_amd._lib import call, load, ptr, stream  # noqa: E402
from tmr_amd.engine import absmax, pack_conv, pack_split_w, pack_split_x, pack_wino  # noqa: E402

FP32_PEAK = 157.3
F16_PEAK = 2516.6  # dense fp16/bf16 MFMA (MI355X_MICROARCH.md)


def timeit(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--units", type=int, default=48)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--H", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    U, H, W, C, N = a.units, a.H, a.H, 512, 2048
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.randn(U, C, H, W, generator=g) * 0.5).to(dev)
    w = (torch.randn(N, C, 3, 3, generator=g) * 0.01).to(dev)
    b = torch.zeros(N, device=dev)
    hw = (torch.randn(N, 5, generator=g) * 0.01).to(dev)
    acc0 = torch.randn(U, N, H, W, device=dev) * 0.1
    part = torch.empty(load().tmr_heads_partials_size(N, U, H, W), device=dev)
    uw, dw = pack_wino(w), pack_conv(w)
    sp = {p: pack_split_w(w, 0, p) for p in ("fp32", "bf16")}
    xmax = absmax(x)
    xs = {p: pack_split_x(x, 3, p, xmax) for p in ("fp32", "bf16")}
    out = torch.empty(U, N, H, W, device=dev)
    ui = torch.arange(U, device=dev, dtype=torch.int32)
    res = {"units": U, "H": H, "K_channels": C, "N": N}
    tiles = ((H + 1) // 2) * ((W + 1) // 2)
    fl_w = 2.0 * 16 * tiles * N * C * U
    fl_d = 2.0 * H * W * N * C * 9 * U
    runs = {
        "wino_heads": (lambda: call("tmr_wino_conv_heads", None, 0, ptr(ui), ptr(x), C, U, H, W, ptr(uw),
                                    ptr(b), N, 1, ptr(hw), ptr(acc0), ptr(part), stream()), fl_w),
        "wino_store": (lambda: call("tmr_wino_conv_store", ptr(x), C, None, None, 0, U, H, W, ptr(uw),
                                    ptr(b), N, 0, None, ptr(out), stream()), fl_w),
        "direct_heads": (lambda: call("tmr_conv_heads", None, 0, ptr(ui), ptr(x), C, U, H, W, ptr(dw),
                                      ptr(b), N, 3, 1, ptr(hw), ptr(acc0), ptr(part), stream()), fl_d),
    }
    for p, terms in (("fp32", 3), ("bf16", 1)):
        pc = {"fp32": 0, "bf16": 1}[p]
        runs[f"split_{p}_heads"] = (
            lambda p=p, pc=pc: call("tmr_split_conv_heads", None, 0, ptr(ui), ptr(xs[p]), C, U, H, W, 3,
                                    pc, ptr(sp[p][0]), ptr(sp[p][1]), ptr(xmax), ptr(b), N, 1, ptr(hw),
                                    ptr(acc0), ptr(part), 2, stream()), fl_d, terms)  # tiled acc0 (engine)
        if p == "bf16":  # bf16 acc0 slab (TMR_SPLIT_INIT_BF16; values are garbage, timing only)
            runs["split_bf16_heads_acc16"] = (
                lambda p=p, pc=pc: call("tmr_split_conv_heads", None, 0, ptr(ui), ptr(xs[p]), C, U, H, W, 3,
                                        pc, ptr(sp[p][0]), ptr(sp[p][1]), ptr(xmax), ptr(b), N, 1, ptr(hw),
                                        ptr(acc0), ptr(part), 2 | 16, stream()), fl_d, terms)
        runs[f"split_{p}_heads_noinit"] = (  # timing only: accumulators start at zero
            lambda p=p, pc=pc: call("tmr_split_conv_heads", None, 0, ptr(ui), ptr(xs[p]), C, U, H, W, 3,
                                    pc, ptr(sp[p][0]), ptr(sp[p][1]), ptr(xmax), ptr(b), N, 1, ptr(hw),
                                    None, ptr(part), 0, stream()), fl_d, terms)
        runs[f"split_{p}_store"] = (
            lambda p=p, pc=pc: call("tmr_split_conv_store", ptr(xs[p]), C, None, None, 0, U, H, W, 3,
                                    pc, ptr(sp[p][0]), ptr(sp[p][1]), ptr(xmax), ptr(b), N, 0, None,
                                    ptr(out), 1, stream()), fl_d, terms)  # tiled out (engine)
        runs[f"split_{p}_xpack"] = (lambda p=p: pack_split_x(x, 3, p, xmax), 0.0, 0)
    # the engine's layout: 3 units per image share the image's acc0 slab
    ui3 = torch.div(torch.arange(U, device=dev, dtype=torch.int32), 3, rounding_mode="floor").to(torch.int32)
    for p, terms, fl16 in (("fp32", 3, 0), ("bf16", 1, 16)):
        pc = {"fp32": 0, "bf16": 1}[p]
        runs[f"split_{p}_heads_e3"] = (
            lambda p=p, pc=pc, fl16=fl16: call("tmr_split_conv_heads", None, 0, ptr(ui3), ptr(xs[p]), C, U, H, W,
                                               3, pc, ptr(sp[p][0]), ptr(sp[p][1]), ptr(xmax), ptr(b), N, 1,
                                               ptr(hw), ptr(acc0), ptr(part), 2 | fl16, stream()), fl_d, terms)
    # the fp-half store at the engine's K = 256 (folded projection): with the
    # broadcast bias-plane initial values (engine) and without
    x256 = x[:, :256].contiguous()
    xs256 = {p: pack_split_x(x256, 3, p, xmax) for p in ("fp32", "bf16")}
    sp256 = {p: pack_split_w(w[:, :256].contiguous(), 256, p) for p in ("fp32", "bf16")}
    fl_256 = fl_d / 2
    for p, terms, fl16 in (("fp32", 3, 0), ("bf16", 1, 8)):
        pc = {"fp32": 0, "bf16": 1}[p]
        for tag, init, flags in (("bplane", acc0, 1 | 2 | 4 | fl16), ("noinit", None, 1 | fl16)):
            runs[f"split_{p}_store256_{tag}"] = (
                lambda p=p, pc=pc, init=init, flags=flags: call(
                    "tmr_split_conv_store", ptr(xs256[p]), 256, None, None, 0, U, H, W, 3, pc, ptr(sp256[p][0]),
                    ptr(sp256[p][1]), ptr(xmax), ptr(b), N, 0, ptr(init) if init is not None else None, ptr(out),
                    flags, stream()), fl_256, terms)
    if os.environ.get("KB_ONLY"):
        runs = {k: v for k, v in runs.items() if k in os.environ["KB_ONLY"].split(",")}
    for name, spec in runs.items():
        fn, fl = spec[0], spec[1]
        fn()
        torch.cuda.synchronize()
        ms = timeit(fn, a.reps)
        r = {"ms": round(ms, 3), "direct_equiv_tflops": round(fl_d / ms / 1e9, 2)}
        if len(spec) == 3:  # split kernel: 16-bit MFMA work = terms x direct FLOPs
            if spec[2]:
                r["mfma16_tflops"] = round(spec[2] * fl / ms / 1e9, 2)
                r["frac_f16_peak"] = round(spec[2] * fl / ms / 1e9 / F16_PEAK, 4)
        else:
            r["executed_tflops"] = round(fl / ms / 1e9, 2)
            r["frac_fp32_peak"] = round(fl / ms / 1e9 / FP32_PEAK, 4)
        res[name] = r
    print(json.dumps(res))


if __name__ == "__main__":
    main()
