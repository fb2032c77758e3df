"""Dump the NMS input of one bench step (per image: the candidates' boxes and
scores in the order tmr_nms sees them) so the pair statistics of the binned
NMS can be studied on the CPU (window sizes, suppressor list lengths).

Run on the GPU box from the repo root:
    python profiles/nms_dump.py --config E --out gpurun_out/nms_E.npz
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (CONFIGS, synthetic inputs)
import tmr_amd as tmr  # noqa: E402
from tmr_amd import host, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="E")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    H = W = 2 * cfg["hf"]
    dev = torch.device("cuda", 0)
    P = synth.reference_state_dict(0, device=dev)
    eng = tmr.TMREngine(P, tmr.PathConfig(precision=cfg.get("precision", "fp32")))
    B, E = cfg["batch"], cfg["E"]
    feats = torch.from_numpy(synth.sam_features(1000, B, bench.CIN, H // 2, W // 2)).to(dev)
    ex, _ = synth.exemplar_set(2000, B, E, H, W, cfg["kmin"], cfg["kmax"])
    boxes = ex.reshape(B * E, 4).astype(np.float32)
    unit_image = np.repeat(np.arange(B), E)
    params = host.peak_params(boxes, H, W, cfg["cls"], eng.cfg.box_reg, False, False)
    with torch.no_grad():
        logits, box, ref, counts = eng._forward_peaks(feats, unit_image, boxes, params)
    c = counts.cpu().numpy()
    lg = logits.cpu().numpy()
    bx = box.cpu().numpy()
    out = {}
    for b in range(B):
        rows = [np.arange(u * H * W, u * H * W + c[u]) for u in range(b * E, (b + 1) * E)]
        r = np.concatenate(rows)
        out[f"boxes_{b}"] = bx[r]
        out[f"scores_{b}"] = lg[r, 0]
    np.savez_compressed(a.out, counts=c, iou=np.float64(cfg["iou"]), **out)
    print("candidates per image:", [int(c[b * E:(b + 1) * E].sum()) for b in range(B)])


if __name__ == "__main__":
    main()
