"""TEST INFRASTRUCTURE ONLY -- end-to-end detection agreement between two sets
of score maps (e.g. the GPU's and the CPU oracle's) for one image.

Peaks and NMS (utils/TM_utils.py:224-323) are discrete functions of the
probability / regression maps.  Two fp32 computations of the same forward that
differ only in summation order (GPU vs CPU, or the reference itself at 1 vs 8
threads: SURVEY.md §4, measured 9e-7 normwise) give maps that differ in the
last ulps, and every DECISION the post-processing takes on a near-tie can flip:

  set flip    a pixel passes `p >= thr` / `pooled == p` on one map only
              (TM_utils.py:253-254);
  order flip  two candidates' scores swap order in NMS's stable descending
              sort (torchvision nms, Appendix B);
  IoU flip    `(double)IoU > iou_threshold` differs for a pair (boxes moved by
              ulps of exp / the regression map).

The post-processing is a deterministic function of these decisions, so with no
flip the two runs keep the same candidates in the same order; with flips the
greedy NMS chain may cascade from the first flipped decision it evaluates.
``compare`` replays both runs through the oracle's C peaks/NMS, finds every
flip and the first divergence of the keep sequences, and reports count delta,
kept-set agreement and matched-box IoU.  The bit-exact contract itself (same
maps -> same detections) is tested separately against the GPU kernels.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

import oracle


def _candidates(maps, boxes, thr):
    """Per unit (idx, logits, boxes, refs) + the exemplar-ordered union with a
    (unit, pixel) identity per row; pixel -1 is the dummy row (TM_utils.py:288-291)."""
    ids, L, B, R = [], [], [], []
    per_unit = []
    for u, ((prob, reg), box) in enumerate(zip(maps, boxes)):
        idx, lg, bx, rf = oracle.peaks_decode(prob, reg, box, thr)
        per_unit.append(set(int(i) for i in idx))
        if lg.shape[0] == 0:
            idx = np.array([-1]); lg, bx, rf = oracle.DUMMY_LOGITS, oracle.DUMMY_BOXES, oracle.DUMMY_REFS
        ids += [(u, int(i)) for i in idx]
        L.append(lg); B.append(bx); R.append(rf)
    return ids, np.concatenate(L), np.concatenate(B), np.concatenate(R), per_unit


def _iou_matrix(b: np.ndarray) -> np.ndarray:
    """fp32 IoU as torchvision's CPU nms evaluates it (Appendix B)."""
    f = np.float32
    x1, y1, x2, y2 = (b[:, i].astype(f) for i in range(4))
    area = (x2 - x1) * (y2 - y1)
    w = np.maximum(f(0), np.minimum(x2[:, None], x2[None]) - np.maximum(x1[:, None], x1[None]))
    h = np.maximum(f(0), np.minimum(y2[:, None], y2[None]) - np.maximum(y1[:, None], y1[None]))
    inter = (w * h).astype(f)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (inter / ((area[:, None] + area[None]).astype(f) - inter)).astype(f)


def compare(maps_a: Sequence, maps_b: Sequence, boxes: Sequence, thr: float, iou: float) -> Dict:
    """maps_*: per unit (prob [H,W], reg [4,H,W]); boxes: per unit exemplar box.
    Returns the agreement report (see module docstring)."""
    ids_a, La, Ba, Ra, pu_a = _candidates(maps_a, boxes, thr)
    ids_b, Lb, Bb, Rb, pu_b = _candidates(maps_b, boxes, thr)
    keep_a = oracle.nms(Ba, La[:, 0], iou)
    keep_b = oracle.nms(Bb, Lb[:, 0], iou)
    kid_a = [ids_a[i] for i in keep_a]
    kid_b = [ids_b[i] for i in keep_b]
    dprob = max(float(np.abs(np.asarray(a[0], np.float64) - b[0]).max()) for a, b in zip(maps_a, maps_b))

    set_flips = sum(len(a ^ b) for a, b in zip(pu_a, pu_b))
    # order / IoU decisions over the candidates both runs have
    pos_b = {k: i for i, k in enumerate(ids_b)}
    common = [i for i, k in enumerate(ids_a) if k in pos_b]
    ia = np.array(common, np.int64)
    ib = np.array([pos_b[ids_a[i]] for i in common], np.int64)
    order_flips = iou_flips = 0
    iou_margin = 0.0
    if ia.size:
        order_flips, iou_flips, iou_margin = oracle.decision_flips(
            Ba[ia], La[ia, 0], ia, Bb[ib], Lb[ib, 0], ib, iou)
    first_div = next((i for i, (x, y) in enumerate(zip(kid_a, kid_b)) if x != y),
                     None if len(kid_a) == len(kid_b) else min(len(kid_a), len(kid_b)))
    sa_set, sb_set = set(kid_a), set(kid_b)
    inter = sa_set & sb_set
    # matched-box IoU: each kept box of run a against the same candidate's kept
    # box in run b, or (kept by a only) its best kept box of run b
    best = np.zeros(len(keep_a))
    if len(keep_a) and len(keep_b):
        kpos_b = {k: i for i, k in enumerate(kid_b)}
        kb = Bb[keep_b]
        for i, k in enumerate(kid_a):
            a = Ba[keep_a[i]][None]
            cand = kb[kpos_b[k]][None] if k in kpos_b else kb
            best[i] = float(np.nan_to_num(_iou_matrix(np.concatenate([a, cand]))[0, 1:], nan=0.0).max())
    same_ids = kid_a == kid_b
    box_diff = float(np.abs(Ba[keep_a] - Bb[keep_b]).max()) if same_ids and len(keep_a) else 0.0
    return dict(
        n_cand=(len(ids_a), len(ids_b)), kept=(len(kid_a), len(kid_b)), count_delta=len(kid_b) - len(kid_a),
        same_kept_ids=same_ids, first_divergence=first_div, jaccard=len(inter) / max(1, len(sa_set | sb_set)),
        matched_iou_min=float(best.min()) if best.size else 1.0,
        matched_iou_mean=float(best.mean()) if best.size else 1.0,
        set_flips=set_flips, order_flips=order_flips, iou_flips=iou_flips, iou_flip_margin=iou_margin,
        max_dprob=dprob, kept_box_max_diff=box_diff, flips=set_flips + order_flips + iou_flips)


def check(rep: Dict) -> None:
    """The contract that holds between two runs of the same forward whose maps
    differ at the ulp level: with no flipped decision the kept candidates are
    the same, in the same order (boxes equal up to the maps' own difference);
    divergence requires a flipped decision."""
    if rep["flips"] == 0:
        assert rep["same_kept_ids"], rep
    if not rep["same_kept_ids"]:
        assert rep["flips"] > 0, rep


def report_line(tag: str, rep: Dict) -> str:
    keys = ("kept", "count_delta", "same_kept_ids", "first_divergence", "jaccard", "matched_iou_min",
            "set_flips", "order_flips", "iou_flips", "max_dprob")
    return tag + " " + " ".join(f"{k}={rep[k]}" for k in keys)


def unit_maps(o: np.ndarray, b: np.ndarray) -> List:
    """[U,1,H,W] logits + [U,4,H,W] regressions -> per unit (prob, reg) with the
    path's sigmoid (tmr_sigmoid_cr)."""
    return [(oracle.sigmoid_cr(o[u, 0]), b[u]) for u in range(o.shape[0])]
