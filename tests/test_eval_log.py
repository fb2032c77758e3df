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


# ---------------------------------------------------------------- COCO AP (log_utils.py:137-205, 379-441)
def _gt(boxes_per_img, crowd=None):
    images = [{"id": i + 1, "height": 100, "width": 100, "file_name": f"{i}.jpg"} for i in range(len(boxes_per_img))]
    anns, aid = [], 1
    for i, bs in enumerate(boxes_per_img):
        for j, (x, y, w, h) in enumerate(bs):
            c = int(bool(crowd and (i, j) in crowd))
            anns.append({"id": aid, "image_id": i + 1, "area": int(w * h), "iscrowd": c,
                         "bbox": [x, y, w, h], "category_id": 1})
            aid += 1
    return {"categories": [{"name": "fg", "id": 1}], "images": images, "annotations": anns}


def _dets(per_img):
    return [{"image_id": i + 1, "category_id": 1, "bbox": list(b), "score": s}
            for i, ds in enumerate(per_img) for b, s in ds]


def _ap(gt, dets):
    ev = eval_log.CocoEvalMaxDets(gt, eval_log.load_res(gt, dets))
    ev.evaluate()
    ev.accumulate()
    ev.summarize()
    return ev


def test_coco_ap_hand_computed():
    # two exact detections of two small GTs: AP 1 at every IoU threshold
    ev = _ap(_gt([[(0, 0, 10, 10), (20, 20, 10, 10)]]), _dets([[((0, 0, 10, 10), .9), ((20, 20, 10, 10), .8)]]))
    assert ev.stats[0] == 1.0 and ev.stats[1] == 1.0 and ev.stats[3] == 1.0
    assert ev.stats[4] == -1 and ev.stats[5] == -1  # no medium / large GT
    # a higher-scored false positive first: precision 1/2 at every recall level
    ev = _ap(_gt([[(0, 0, 10, 10)]]), _dets([[((50, 50, 10, 10), .9), ((0, 0, 10, 10), .8)]]))
    assert ev.stats[0] == 0.5 and ev.stats[8] == 1.0
    # IoU 90/110 = 0.818: matched for t = .50 ... .80 (7 of 10 thresholds)
    ev = _ap(_gt([[(0, 0, 10, 10)]]), _dets([[((1, 0, 10, 10), .7)]]))
    # (precision tp / (fp + tp + eps) = 1 / (1 + 2^-52) < 1 for a single detection, as pycocotools)
    assert abs(ev.stats[0] - 0.7) < 1e-12 and abs(ev.stats[1] - 1.0) < 1e-12 and abs(ev.stats[2] - 1.0) < 1e-12
    # a detection inside a crowd region is ignored, not a false positive
    gt = _gt([[(0, 0, 10, 10), (40, 40, 50, 50)]], crowd={(0, 1)})
    ev = _ap(gt, _dets([[((0, 0, 10, 10), .5), ((45, 45, 10, 10), .9)]]))
    assert abs(ev.stats[0] - 1.0) < 1e-12
    # no results: pycocotools' loadRes indexes anns[0]
    with pytest.raises(IndexError):
        eval_log.load_res(gt, [])


def _literal_match(ious, gtIg, iscrowd, gt_ids, dt_ids, thrs):
    """COCOeval.evaluateImg's matching loop transcribed literally."""
    T, D, G = len(thrs), ious.shape[0], ious.shape[1]
    gtm, dtm, dtIg = np.zeros((T, G)), np.zeros((T, D)), np.zeros((T, D))
    for tind, t in enumerate(thrs):
        for dind in range(D):
            iou = min([t, 1 - 1e-10])
            m = -1
            for gind in range(G):
                if gtm[tind, gind] > 0 and not iscrowd[gind]:
                    continue
                if m > -1 and gtIg[m] == 0 and gtIg[gind] == 1:
                    break
                if ious[dind, gind] < iou:
                    continue
                iou = ious[dind, gind]
                m = gind
            if m == -1:
                continue
            dtIg[tind, dind] = gtIg[m]
            dtm[tind, dind] = gt_ids[m]
            gtm[tind, m] = dt_ids[dind]
    return gtm, dtm, dtIg


@pytest.mark.parametrize("seed", range(6))
def test_coco_matching_equals_literal_loop(seed):
    """Random clustered boxes (ties, crowds, every area range): the
    vectorised matching equals the literal transcription per image and
    area range; AP/AR stay in [0, 1]."""
    rng = np.random.default_rng(seed)
    gts, dts, crowd = [], [], set()
    for i in range(4):
        n = int(rng.integers(0, 12))
        bs = [(float(rng.integers(0, 60)), float(rng.integers(0, 60)), float(rng.choice([4, 8, 40, 120])),
               float(rng.choice([4, 8, 40, 120]))) for _ in range(n)]
        gts.append(bs)
        for j in range(n):
            if rng.random() < 0.15:
                crowd.add((i, j))
        ds = []
        for _ in range(int(rng.integers(0, 20))):
            if bs and rng.random() < 0.7:
                x, y, w, h = bs[int(rng.integers(0, len(bs)))]
                b = (x + float(rng.integers(-3, 4)), y + float(rng.integers(-3, 4)), w, h)
            else:
                b = (float(rng.integers(0, 90)), float(rng.integers(0, 90)), 8.0, 8.0)
            ds.append((b, float(rng.choice([0.3, 0.5, 0.5, 0.9]))))  # tied scores
        dts.append(ds)
    gt = _gt(gts, crowd)
    if not any(dts):
        dts[0] = [((0.0, 0.0, 5.0, 5.0), 0.5)]
    ev = _ap(gt, _dets(dts))
    p = ev.params
    for a_i, arng in enumerate(p.areaRng):
        for i_i, img in enumerate(p.imgIds):
            e = ev.evalImgs[a_i * len(p.imgIds) + i_i]
            g = ev._gts.get((img, 1), [])
            d = ev._dts.get((img, 1), [])
            if e is None:
                assert not g and not d
                continue
            g_ign = [1 if (x["ignore"] or x["area"] < arng[0] or x["area"] > arng[1]) else 0 for x in g]
            gi = np.argsort(g_ign, kind="mergesort")
            gs = [g[k] for k in gi]
            di = np.argsort([-x["score"] for x in d], kind="mergesort")
            ds_ = [d[k] for k in di]
            if not gs or not ds_:
                continue
            ious = eval_log.bbox_iou([x["bbox"] for x in ds_], [x["bbox"] for x in gs],
                                     [x["iscrowd"] for x in gs])
            gtm, dtm, dtIg = _literal_match(ious, [g_ign[k] for k in gi], [x["iscrowd"] for x in gs],
                                            [x["id"] for x in gs], [x["id"] for x in ds_], p.iouThrs)
            np.testing.assert_array_equal(e["gtMatches"], gtm)
            np.testing.assert_array_equal(e["dtMatches"], dtm)
            a = np.array([x["area"] < arng[0] or x["area"] > arng[1] for x in ds_]).reshape(1, -1)
            np.testing.assert_array_equal(e["dtIgnore"], np.logical_or(dtIg, (dtm == 0) & np.repeat(a, 10, 0)))
    s = ev.stats
    assert all(v == -1 or 0 <= v <= 1 for v in s)


def test_get_ap_scores_on_generated_files(tmp_path, monkeypatch):
    """Get_AP_scores over the COCO files the restated generator writes for
    the golden case (values parity-unpinned: pycocotools absent)."""
    g = json.load(open(GOLDEN))
    real = os.listdir
    monkeypatch.setattr(eval_log.os, "listdir", lambda p: sorted(real(p)))
    batch, L, B, R = _inputs(g)
    eval_log.image_info_collector(str(tmp_path), "test", batch, L, B, R)
    eval_log.coco_style_annotation_generator(str(tmp_path), "test")
    ap, ap50, ap75 = eval_log.Get_AP_scores(str(tmp_path), "test")
    assert 0.0 <= ap <= ap50 <= 100.0 and 0.0 <= ap75 <= ap50
