"""Where the module path's (config A, `bench.py --path module`) host time
goes: the bench's per-image call sequence (demo.py:106-130) with host clock
stamps around the points where the GPU waits for the host -- each graph
replay's launch and each host sync (Get_pred_boxes' counts, the NMS size).
A sync returns when the GPU has drained, so (next launch - sync return) is
GPU idle time spent in Python.  Profiling only: the stamps come from
wrappers installed around engine methods by this script.

    python profiles/module_phases.py [--steps 64]

The workload is bench.py's config A: one image (SAM features 256x64x64),
3 exemplars (k 7..15), cls 0.7, IoU 0.5, the same image every step.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

tmr = load_package()
from tmr_amd import engine as E_, synth  # noqa: E402

STAMPS = []


def stamp(tag):
    STAMPS.append((tag, time.perf_counter()))


class _Counts:
    def __init__(self, t):
        self.t = t

    def cpu(self):
        stamp("sync0")
        r = self.t.cpu()
        stamp("sync1")
        return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--cprofile", default="", help="write a cProfile of the timed steps to this file")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from types import SimpleNamespace
    CIN, EMB = 256, 512
    margs = SimpleNamespace(emb_dim=EMB, fusion=True, ablation_no_box_regression=False, encoder="original",
                            feature_upsample=True, no_matcher=False, template_type="roi_align", squeeze=False,
                            decoder_num_layer=1, decoder_kernel_size=3, modeltype="matching_net",
                            backbone="features", num_channels=CIN, precision="fp32")
    P = synth.reference_state_dict(0, device=dev)
    model = tmr.build_model(margs)
    model.load_state_dict(P, strict=True)
    model = model.to(dev).eval()
    B, E = a.steps, 3
    feats = torch.from_numpy(synth.sam_features(1000, 1, CIN, 64, 64)).to(dev)
    ex, _ = synth.exemplar_set(2000, 1, E, 128, 128, 7, 15)
    dummy = {"regression_ablation_b": False, "regression_ablation_c": False}

    peaks0, nms0, replay0 = E_.TMREngine.peaks, E_.TMREngine.nms, E_._DetectGraph.replay

    def peaks(*args, **kw):
        r = peaks0(*args, **kw)
        return r[:3] + (_Counts(r[3]),) + r[4:]

    def nms(*args, **kw):
        stamp("nms0")
        r = nms0(*args, **kw)
        stamp("nms1")
        return r

    def replay(self, *args, **kw):
        stamp("replay0")
        r = replay0(self, *args, **kw)
        stamp("replay1")
        return r

    E_.TMREngine.peaks = staticmethod(peaks)
    E_.TMREngine.nms = staticmethod(nms)
    E_._DetectGraph.replay = replay

    def image(b):
        stamp("img")
        image_t = feats[0:1]  # a fresh view per image, as bench.py's loop makes
        ex_d = torch.from_numpy(ex[0]).pin_memory().to(dev, non_blocking=True)
        pl, pb, pr = [], [], []
        for exemplar in [[ex_d[e].unsqueeze(0)] for e in range(E)]:
            stamp("fwd")
            po, preg, _, _ = model(image_t, exemplar)
            stamp("gpb")
            _l, _b, _r = tmr.Get_pred_boxes(po, preg, exemplar, dummy, 0.7, True)
            stamp("gpb1")
            pl.append(_l[0]); pb.append(_b[0]); pr.append(_r[0])
        stamp("cat")
        L_, _, _ = tmr.NMS([torch.concat(pl)], [torch.concat(pb)], [torch.concat(pr)], 0.5)
        stamp("end")
        return L_

    with torch.no_grad():
        for b in range(4):  # warm: graphs captured
            image(b)
        torch.cuda.synchronize()
        STAMPS.clear()
        prof = None
        if a.cprofile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        for b in range(B):
            image(b)
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
        if prof is not None:
            prof.disable()
            import pstats
            with open(a.cprofile, "w") as fh:
                pstats.Stats(prof, stream=fh).sort_stats("tottime").print_stats(45)
    # intervals between consecutive stamps, by (from, to) tag pair
    agg = {}
    for (t1, a1), (t2, a2) in zip(STAMPS, STAMPS[1:]):
        k = f"{t1}->{t2}"
        agg.setdefault(k, []).append(1e6 * (a2 - a1))
    rows = {k: {"n": len(v), "mean_us": round(float(np.mean(v)), 1), "sum_us_per_image": round(float(np.sum(v)) / B, 1)}
            for k, v in agg.items()}
    print(json.dumps({"ms_per_image": round(1e3 * total / B, 4), "intervals": rows}, indent=1))


if __name__ == "__main__":
    main()
