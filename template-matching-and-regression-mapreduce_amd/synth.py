"""Synthetic, portable inputs for the TMR hot path.

* SAM-like features: counter-based splitmix64 -> Box-Muller normals, then a
  per-pixel LayerNorm over channels (SAM's neck ends in LayerNorm2d,
  models/backbone/sam/sam_ViT.py:88-104).
* Exemplar boxes sized so the RoIAlign template is exactly k x k on the
  matching map: x1 = (i + 0.25)/W, x2 = x1 + (k - 0.5)/W, which makes
  ceil(x2*W) - floor(x1*W) = k (models/template_matching.py:66-73).

Pure numpy with explicit uint64 arithmetic so every host reproduces the same
values without torch's RNG.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """n outputs of splitmix64 at counters seed*2^32 + stream*2^48 + [1..n]."""
    with np.errstate(over="ignore"):
        base = np.uint64((int(seed) * (1 << 32) + int(stream) * (1 << 48)) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """float64 uniforms in [0, 1)."""
    return (splitmix64(seed, n, stream) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def normal(seed: int, shape, stream: int = 0) -> np.ndarray:
    n = int(np.prod(shape))
    m = (n + 1) // 2
    u = uniform(seed, 2 * m, stream)
    u1, u2 = 1.0 - u[:m], u[m:]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])[:n]
    return z.astype(np.float32).reshape(shape)


def sam_features(seed: int, B: int, C: int = 256, H: int = 64, W: int = 64) -> np.ndarray:
    """[B,C,H,W] fp32, standard normal then LayerNorm over C (eps 1e-6)."""
    x = normal(seed, (B, C, H, W)).astype(np.float64)
    mu = x.mean(axis=1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=1, keepdims=True)
    return ((x - mu) / np.sqrt(var + 1e-6)).astype(np.float32)


def exemplar_box(k: int, H: int, W: int, iy: int, ix: int, kw: int | None = None) -> np.ndarray:
    """Normalised xyxy box giving a k x kw (odd) template on an H x W map."""
    kw = k if kw is None else kw
    x1 = (ix + 0.25) / W
    y1 = (iy + 0.25) / H
    return np.array([x1, y1, x1 + (kw - 0.5) / W, y1 + (k - 0.5) / H], np.float32)


def exemplar_set(seed: int, B: int, E: int, H: int, W: int, kmin: int = 3, kmax: int = 15):
    """[B,E,4] boxes with odd template sizes uniform over {kmin..kmax} and
    uniform positions, plus the [B,E] array of sizes."""
    ks_choices = np.arange(kmin, kmax + 1, 2)
    u = uniform(seed, 3 * B * E, stream=7).reshape(B, E, 3)
    ks = ks_choices[np.minimum((u[..., 0] * len(ks_choices)).astype(int), len(ks_choices) - 1)]
    boxes = np.zeros((B, E, 4), np.float32)
    for b in range(B):
        for e in range(E):
            k = int(ks[b, e])
            iy = int(u[b, e, 1] * (H - k + 1))
            ix = int(u[b, e, 2] * (W - k + 1))
            boxes[b, e] = exemplar_box(k, H, W, iy, ix)
    return boxes, ks


def reference_state_dict(seed: int, cin: int = 256, emb: int = 512, num_layers: int = 1,
                         k: int = 3, obj_bias: float = 0.0, device="cpu"):
    """Random weights with the reference initialisation (regression_head.py:19-24:
    N(0, 0.01) conv weights, zero bias; nn.Conv2d default for input_proj;
    matcher.scale = 1.0), under the reference state_dict keys (fusion, box
    regression).  ``obj_bias`` optionally shifts the objectness bias."""
    import math

    import torch

    g = torch.Generator().manual_seed(seed)
    P = {"matcher.scale": torch.tensor([1.0])}
    bound = 1.0 / math.sqrt(cin)
    P["input_proj.0.weight"] = (torch.rand(emb, cin, 1, 1, generator=g) * 2 - 1) * bound
    P["input_proj.0.bias"] = (torch.rand(emb, generator=g) * 2 - 1) * bound
    d = 2 * emb
    for pre in ("decoder_b", "decoder_o"):
        for l in range(num_layers):
            P[f"{pre}.layer.{2 * l}.weight"] = torch.randn(d, d, k, k, generator=g) * 0.01
            P[f"{pre}.layer.{2 * l}.bias"] = torch.zeros(d)
    P["objectness_head.head.0.weight"] = torch.randn(1, d, 1, 1, generator=g) * 0.01
    P["objectness_head.head.0.bias"] = torch.full((1,), float(obj_bias))
    P["ltrbs_head.head.0.weight"] = torch.randn(4, d, 1, 1, generator=g) * 0.01
    P["ltrbs_head.head.0.bias"] = torch.zeros(4)
    return {k_: v.float().to(device) for k_, v in P.items()}


def sam_features_device(seeds, C: int = 256, H: int = 64, W: int = 64, device="cuda"):
    """Device-side counterpart of sam_features for the streaming driver: per
    seed a standard normal [C,H,W] from a seeded torch generator on `device`,
    LayerNorm over C (eps 1e-6).  Not bit-identical to sam_features (a
    different PRNG); used where the features are only workload, not a
    parity input."""
    import torch

    out = torch.empty((len(seeds), C, H, W), device=device, dtype=torch.float32)
    g = torch.Generator(device=device)
    for i, s in enumerate(seeds):
        g.manual_seed(int(s))
        out[i].normal_(generator=g)
    mu = out.mean(dim=1, keepdim=True)
    var = (out - mu).pow(2).mean(dim=1, keepdim=True)
    return (out - mu) / torch.sqrt(var + 1e-6)
