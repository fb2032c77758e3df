"""Eval bookkeeping (utils/log_utils.py:21-136, 214-309).

CPU: the restatement writes byte-identical files (per-image JSONs, COCO GT /
prediction files, MAE_RMSE text) and the same MAE/RMSE as the reference
log_utils.py on the golden case (tests/golden/evallog_cases.json, made by
oracle/make_golden_evallog.py running the reference).  GPU: kept detections
straight from TMREngine.detect produce the same per-image counts as the
oracle pipeline through the same bookkeeping.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_REPO, os.path.join(_REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
from tmr_import import load_package  # noqa: E402

load_package()
import oracle  # noqa: E402
from tmr_amd import eval_log, synth  # noqa: E402

GOLDEN = os.path.join(_REPO, "tests", "golden", "evallog_cases.json")


def _inputs(g):
    b = dict(g["batch"])
    b["img_size"] = torch.tensor(b["img_size"])
    b["orig_boxes"] = [np.array(x, np.float32) for x in b["orig_boxes"]]
    b["orig_exemplars"] = [np.array(x, np.float32) for x in b["orig_exemplars"]]
    t = lambda xs: [torch.tensor(x, dtype=torch.float32) for x in xs]  # noqa: E731
    return b, t(g["logits"]), t(g["boxes"]), t(g["refs"])


def _files(d):
    out = {}
    for root, _, fs in os.walk(d):
        for f in fs:
            p = os.path.join(root, f)
            out[os.path.relpath(p, d)] = open(p).read()
    return out


def test_eval_files_match_reference(tmp_path, monkeypatch):
    g = json.load(open(GOLDEN))
    real = os.listdir
    monkeypatch.setattr(eval_log.os, "listdir", lambda p: sorted(real(p)))
    batch, L, B, R = _inputs(g)
    eval_log.image_info_collector(str(tmp_path), "test", batch, L, B, R)
    eval_log.coco_style_annotation_generator(str(tmp_path), "test")
    mae, rmse = eval_log.Get_MAE_RMSE(str(tmp_path), "test")
    got = _files(str(tmp_path))
    assert sorted(got) == sorted(g["files"])
    for k in got:
        assert got[k] == g["files"][k], k
    assert mae == g["mae"] and float(rmse) == g["rmse"]


def test_refinery_edges():
    # threshold 0 keeps score-0 rows (the dummy), drops negatives
    lg = torch.tensor([[0.0, 0.0], [-1e-9, 0.0], [0.5, 0.0]])
    bx = torch.tensor([[0.0, 0.0, 1e-14, 1e-14], [0.1, 0.1, 0.2, 0.2], [0.25, 0.5, 0.75, 1.0]])
    rf = torch.tensor([[0.0, 0.0], [0.15, 0.15], [0.5, 0.75]])
    l, b, p = eval_log.pred_refinery(lg, bx, rf, [100, 10])
    assert l == [[0.0, 0.0], [0.5, 0.0]]
    assert b == [[0, 0, 0, 0], [25, 5, 50, 5]]
    assert p == [[0, 0], [50, 8]]


DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


@pytest.mark.gpu
def test_counts_from_gpu_detections(tmp_path):
    from tmr_amd import PathConfig, TMREngine

    P = oracle.reference_weights(0, cin=32, emb=32)
    P["objectness_head.head.0.bias"] = torch.tensor([0.4])
    feats = synth.sam_features(21, 3, 32, 12, 12)
    ex, _ = synth.exemplar_set(22, 3, 2, 24, 24, 3, 7)
    eng = TMREngine({k: v.to(DEV) for k, v in P.items()}, PathConfig(emb_dim=32))
    L, Bx, R = eng.detect(torch.from_numpy(feats).to(DEV), ex, cls_ths=0.5, iou_threshold=0.5)
    ol, ob, orr = [], [], []
    for b in range(3):
        ls, bs, rs = [], [], []
        for e in range(2):
            exm = [torch.from_numpy(ex[b, e:e + 1])]
            o, bb, _, _ = oracle.forward_torch(torch.from_numpy(feats[b:b + 1]), exm, P)
            prob = oracle.sigmoid_cr(o[0][0, 0].numpy())
            l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [bb[0][0].numpy()], exm, 0.5)
            ls.append(l_[0]); bs.append(b_[0]); rs.append(r_[0])
        l2, b2, r2 = oracle.nms_lists([np.concatenate(ls)], [np.concatenate(bs)], [np.concatenate(rs)], 0.5)
        ol.append(torch.from_numpy(l2[0])); ob.append(torch.from_numpy(b2[0])); orr.append(torch.from_numpy(r2[0]))
    batch = {"img_name": [f"i{b}.jpg" for b in range(3)], "img_url": [""] * 3, "img_id": [1, 2, 3],
             "img_size": torch.tensor([[512, 384]] * 3),
             "orig_boxes": [np.array([[0, 0, 10, 10]] * (b + 2), np.float32) for b in range(3)],
             "orig_exemplars": [np.array([[0, 0, 10, 10]], np.float32)] * 3}
    res = {}
    for name, (l, bx, r) in {"gpu": (L, Bx, R), "oracle": (ol, ob, orr)}.items():
        d = str(tmp_path / name)
        eval_log.image_info_collector(d, "t", batch, l, bx, r)
        eval_log.coco_style_annotation_generator(d, "t")
        res[name] = (eval_log.Get_MAE_RMSE(d, "t"),
                     sorted(open(os.path.join(d, "MAE_RMSE_t.txt")).read().splitlines()))
    assert res["gpu"] == res["oracle"]
