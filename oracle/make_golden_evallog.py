"""TEST INFRASTRUCTURE ONLY -- golden files for the eval bookkeeping (§8f f2).

Imports the reference's utils/log_utils.py from /root/reference and runs
image_info_collector -> coco_style_annotation_generator -> Get_MAE_RMSE on
seeded synthetic predictions (incl. an image whose only row is the
Get_pred_boxes dummy, negative scores, boxes crossing the image border,
sub-pixel sizes), then stores the inputs and every file it wrote in
tests/golden/evallog_cases.json.

Stubs (modules absent from this image; none of them computes anything the
fixtures record): cv2, matplotlib.pyplot, torchmetrics.detection,
pycocotools.cocoeval; pycocotools.coco.COCO is replaced by the minimal index
Get_MAE_RMSE needs (images in file order, annotation ids per image id, as
pycocotools' getImgIds / getAnnIds / loadImgs).  os.listdir is sorted in
both this generator and the test, so the file order is fixed.

Usage (this container only):  PYTHONDONTWRITEBYTECODE=1 python oracle/make_golden_evallog.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference/utils/log_utils.py"


class _Coco:
    def __init__(self, path):
        with open(path) as fh:
            d = json.load(fh)
        self.imgs = {im["id"]: im for im in d["images"]}
        self.ia = {}
        for a in d["annotations"]:
            self.ia.setdefault(a["image_id"], []).append(a["id"])

    def getImgIds(self):
        return list(self.imgs.keys())

    def getAnnIds(self, ids):
        return [a for i in ids for a in self.ia.get(i, [])]

    def loadImgs(self, ids):
        return [self.imgs[i] for i in ids]


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def load_ref():
    _stub("cv2")
    _stub("matplotlib"); _stub("matplotlib.pyplot")
    _stub("torchmetrics"); _stub("torchmetrics.detection", MeanAveragePrecision=object)
    _stub("pycocotools"); _stub("pycocotools.coco", COCO=_Coco)
    _stub("pycocotools.cocoeval", COCOeval=object)
    spec = importlib.util.spec_from_file_location("ref_log_utils", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_inputs(seed=0):
    rng = np.random.default_rng(seed)
    B = 4
    batch = {"img_name": [f"img_{i}.jpg" for i in range(B)], "img_url": [f"/data/img_{i}.jpg" for i in range(B)],
             "img_id": [101 + 7 * i for i in range(B)],
             "img_size": torch.tensor([[1920, 1280], [640, 480], [1024, 1024], [333, 517]]),
             "orig_boxes": [], "orig_exemplars": []}
    L, Bx, R = [], [], []
    for i in range(B):
        W, H = batch["img_size"][i].tolist()
        n = int(rng.integers(1, 9))
        xy = rng.uniform(0, 1, (n, 2)) * [W, H]
        wh = rng.uniform(2, 80, (n, 2))
        batch["orig_boxes"].append(np.concatenate([xy, xy + wh], 1).astype(np.float32))
        batch["orig_exemplars"].append(batch["orig_boxes"][-1][:3].copy())
        if i == 2:  # Get_pred_boxes dummy row (TM_utils.py:288-291)
            L.append(torch.tensor([[0.0, 0.0]])); Bx.append(torch.tensor([[0.0, 0.0, 1e-14, 1e-14]]))
            R.append(torch.tensor([[0.0, 0.0]])); continue
        k = int(rng.integers(3, 12))
        c = rng.uniform(-0.05, 1.05, (k, 2)).astype(np.float32)
        s = rng.uniform(0.0005, 0.2, (k, 2)).astype(np.float32)
        box = np.concatenate([c - s / 2, c + s / 2], 1).astype(np.float32)
        sc = rng.uniform(-0.1, 1, k).astype(np.float32)
        sc[0] = 0.0
        L.append(torch.from_numpy(np.stack([sc, np.zeros(k, np.float32)], 1)))
        Bx.append(torch.from_numpy(box)); R.append(torch.from_numpy(c))
    return batch, L, Bx, R


def main():
    ref = load_ref()
    real_listdir = os.listdir
    os.listdir = lambda p: sorted(real_listdir(p))
    batch, L, Bx, R = make_inputs()
    with tempfile.TemporaryDirectory() as d:
        ref.image_info_collector(d, "test", batch, L, Bx, R)
        ref.coco_style_annotation_generator(d, "test")
        mae, rmse = ref.Get_MAE_RMSE(d, "test")
        files = {}
        for root, _, fs in os.walk(d):
            for f in fs:
                p = os.path.join(root, f)
                files[os.path.relpath(p, d)] = open(p).read()
    os.listdir = real_listdir
    out = {"batch": {k: (v.tolist() if isinstance(v, torch.Tensor) else
                         [x.tolist() for x in v] if k.startswith("orig") else v) for k, v in batch.items()},
           "logits": [t.tolist() for t in L], "boxes": [t.tolist() for t in Bx], "refs": [t.tolist() for t in R],
           "mae": mae, "rmse": float(rmse), "files": files}
    dst = os.path.join(REPO, "tests", "golden", "evallog_cases.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", dst, sorted(files), mae, rmse)


if __name__ == "__main__":
    main()
