"""Normwise error of the 3-term MFMA correlation against the fp32 VALU kernel
(same engine, same templates) per template size: the template split scheme's
precision (TH_BITS; TMR_LIB_VARIANT selects the library).  The VALU kernel's
own error (fp32 FMA chains of <= 961 taps) is ~1e-7, far below the contract.

    python profiles/xcorr_error.py
"""
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

dev = torch.device("cuda:0")
P = {k: v.to(dev) for k, v in synth.reference_state_dict(0).items()}
eng = tmr.TMREngine(P, tmr.PathConfig())
worst = {}
for seed, (H, kk) in enumerate([(64, (3, 9)), (128, (11, 15)), (192, (21, 31))]):
    g = torch.Generator(device=dev).manual_seed(seed)
    B, E = 2, 3
    fp = torch.randn((B, 512, H, H), device=dev, generator=g)
    ex, ks = synth.exemplar_set(seed, B, E, H, H, kk[0], kk[1])
    ui = np.repeat(np.arange(B), E)
    out = {}
    for algo in ("valu", "mfma"):
        eng.xcorr_algo = algo
        ftm, _ = eng.match(fp, ui, ex.reshape(-1, 4))
        out[algo] = ftm.double()
    d = (out["mfma"] - out["valu"]).abs().amax(dim=(1, 2, 3)) / out["valu"].abs().amax(dim=(1, 2, 3))
    worst[f"{H}:{kk[0]}-{kk[1]}"] = float(d.max())
print(json.dumps({"variant": os.environ.get("TMR_LIB_VARIANT", "base"), "normwise": worst}))
