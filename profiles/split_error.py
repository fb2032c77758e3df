"""Normwise error of the split decoder conv (tmr_split_conv, fp32
contract) against an fp64 torch conv on decoder-shaped inputs: the weights'
split scheme's precision (VARIANT selects the library, TMR_LIB_VARIANT)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

load_package()
from tmr_amd.engine import conv2d_split  # noqa: E402

dev = torch.device("cuda:0")
worst = {}
for seed, (C, N, H, W) in enumerate([(1024, 512, 32, 32), (512, 2048, 24, 40), (257, 256, 33, 17)]):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((2, C, H, W), generator=g, dtype=torch.float64)
    w = torch.randn((N, C, 3, 3), generator=g, dtype=torch.float64) * 0.01
    b = torch.randn(N, generator=g, dtype=torch.float64) * 0.01
    ref = torch.nn.functional.conv2d(x, w, b, padding=1)
    got = conv2d_split(x.float().to(dev), w.float().to(dev), b.float().to(dev), False, "fp32").cpu().double()
    # fp32-rounded inputs are the reference's inputs too
    ref32 = torch.nn.functional.conv2d(x.float().double(), w.float().double(), b.float().double(), padding=1)
    err = float((got - ref32).abs().max() / ref32.abs().max())
    worst[f"{C}x{N}"] = err
print(json.dumps({"variant": os.environ.get("TMR_LIB_VARIANT", "base"), "normwise": worst}))
