"""Drop-in post-processing (reference: utils/TM_utils.py:9-18, 224-377).

``Get_pred_boxes`` and ``NMS`` keep the reference's signatures, argument
conventions and list-of-per-image-tensors results; the peak finder, decode
and NMS run in libtmr.so (tmr_peaks_decode, tmr_nms).  Like the reference,
each call syncs once to learn the variable-length result sizes.
"""
from __future__ import annotations

import numpy as np
import torch

from . import host
from ._lib import TMRError, call, ptr, require_gpu, stream
from .engine import TMREngine
from .template_matching import _box_host


def calc_area(box):
    """TM_utils.py:9-11."""
    x1, y1, x2, y2 = box
    return (x2 - x1) * (y2 - y1)


def map_normalization(img):
    """TM_utils.py:325-335: min-max scaling of a map (display helper; torch
    ops on the tensor's own device, numpy for arrays, as the reference)."""
    if torch.is_tensor(img):
        maxv, minv = torch.max(img), torch.min(img)
    else:
        maxv, minv = np.max(img), np.min(img)
    return (img - minv) / (maxv - minv + 1e-14)


def custom_shape_3x3_maxpool2d(x: torch.Tensor, kernel: list) -> torch.Tensor:
    """TM_utils.py:337-361 on the GPU (tmr_maxpool3x3): the max over the
    3x3 neighbourhood positions where ``kernel`` is 1 (zero padding, as
    F.unfold), [N,C,H,W] -> [N,C,H,W] in x's dtype (the max is exact)."""
    require_gpu(x, "x")
    if x.dim() != 4:
        raise TMRError(f"custom_shape_3x3_maxpool2d: expected [N,C,H,W], got {tuple(x.shape)}")
    k = np.asarray(kernel, dtype=bool).reshape(3, 3)
    mask = int(sum(1 << (3 * r + c) for r in range(3) for c in range(3) if k[r, c]))
    if mask == 0:  # torch.max over an empty selection raises too
        raise TMRError("custom_shape_3x3_maxpool2d: the kernel selects no position")
    xf = x.detach().float().contiguous()
    N, C, H, W = xf.shape
    out = torch.empty_like(xf)
    call("tmr_maxpool3x3", ptr(xf), N * C, H, W, mask, ptr(out), stream())
    return out if x.dtype == torch.float32 else out.to(x.dtype)


def Make_Template_size_predictions(centers):
    """TM_utils.py:13-18: zero regressions (box = exemplar size)."""
    xy = torch.zeros_like(centers)
    wh = torch.zeros_like(centers)
    return torch.concat([xy, wh], dim=1)


def adaptive_kernel_generater(ex_size, pred_size):
    """TM_utils.py:363-377 (fp32 comparisons, as with 0-d tensors)."""
    ex_h, ex_w = [float(v) for v in ex_size]
    return host.mask_to_kernel(host.adaptive_mask(ex_h, ex_w, int(pred_size[0]), int(pred_size[1])))


_DUMMY: "dict[tuple, tuple]" = {}


def _dummy(dtype, device):
    """The empty-unit rows of TM_utils.py:288-291, fresh tensors per call.
    Cloned on the device from a cached copy: building them from Python
    values is a pageable host->device copy, which waits for the stream."""
    key = (dtype, str(device))
    d = _DUMMY.get(key)
    if d is None:
        d = _DUMMY[key] = (torch.tensor([[0.0, 0.0]], dtype=dtype, device=device),
                           torch.tensor([[0.0, 0.0, 1e-14, 1e-14]], dtype=dtype, device=device),
                           torch.tensor([[0.0, 0.0]], dtype=dtype, device=device))
    return tuple(t.clone() for t in d)


def Get_pred_boxes(pred_objectness, pred_regressions, exemplars, batch, cls_ths=0.1, box_reg=True,
                   input_is_prob=False):
    """TM_utils.py:224-305.  pred_objectness: list over levels of [B,1,H,W]
    logits; pred_regressions: list of [B,4,H,W] (or None entries).
    Returns (pred_logits, pred_boxes, ref_points): lists over images.  An
    image's candidate rows are views into this call's own (fresh) peak
    buffers, as the reference's boolean-index results are fresh tensors.
    ``input_is_prob`` (extension) feeds probability maps instead of logits,
    the form the bit-exact contract is stated on."""
    dtype = pred_objectness[-1].dtype
    device = pred_objectness[-1].device
    require_gpu(pred_objectness[0], "pred_objectness")
    B = len(pred_objectness[0])
    boxes = np.stack([_box_host(exemplars[b][0]) for b in range(B)])
    ab_b = bool(batch["regression_ablation_b"])
    ab_c = bool(batch["regression_ablation_c"])
    per_level = []
    for level in range(len(pred_objectness)):
        o = pred_objectness[level]
        H, W = o.shape[-2:]
        reg = pred_regressions[level] if (box_reg and pred_regressions is not None) else None
        params = host.peak_params(boxes, H, W, cls_ths, box_reg, ab_b, ab_c)
        logits, box, ref, counts, _ = TMREngine.peaks(o, reg, params, input_is_prob, want_prob=False)
        counts = counts.cpu().numpy()  # torch.where's sync (TM_utils.py:254)
        cap = H * W
        per_level.append([(logits[b * cap:b * cap + counts[b]], box[b * cap:b * cap + counts[b]],
                           ref[b * cap:b * cap + counts[b]]) for b in range(B)])
        if level == 0:  # an empty unit's row 0 holds the dummy row (tmr_peaks_decode)
            lv0 = (logits, box, ref, cap)
    pred_logits, pred_boxes, ref_points = [], [], []
    for b in range(B):
        parts = [lv[b] for lv in per_level]
        if len(parts) == 1:
            lg, bx, rf = parts[0]
        else:
            lg = torch.cat([p[0] for p in parts]); bx = torch.cat([p[1] for p in parts])
            rf = torch.cat([p[2] for p in parts])
        if lg.shape[0] == 0:  # every level empty: the dummy row, fresh 1-row tensors as the
            # reference's (TM_utils.py:288-291): cloned on the device (no sync), so a kept
            # dummy does not hold the call's [U*H*W] peak buffers alive
            lg, bx, rf = (tuple(t[b * lv0[3]:b * lv0[3] + 1].clone() for t in lv0[:3])
                          if dtype == torch.float32 else _dummy(dtype, device))
        pred_logits.append(lg); pred_boxes.append(bx); ref_points.append(rf)
    return pred_logits, pred_boxes, ref_points


def _nms_lists(pred_logits, pred_boxes, ref_points, iou_threshold, want_keep=False):
    G = len(pred_logits)
    ns = np.array([int(x.shape[0]) for x in pred_logits], np.int64)
    live = [g for g in range(G) if ns[g] > 0]
    outs = {}
    if live:
        dev = pred_logits[live[0]].device
        for g in live:
            require_gpu(pred_logits[g], "pred_logits")
        if len(live) == 1:  # one list (the demo.py call form): no concatenation copy
            g0 = live[0]
            lg, bx, rf = (pred_logits[g0].float().contiguous(), pred_boxes[g0].float().contiguous(),
                          ref_points[g0].float().contiguous())
        else:
            lg = torch.cat([pred_logits[g].float() for g in live]).contiguous()
            bx = torch.cat([pred_boxes[g].float() for g in live]).contiguous()
            rf = torch.cat([ref_points[g].float() for g in live]).contiguous()
        counts_h = ns[live]
        unit_off = np.zeros(len(live), np.int64)
        unit_off[1:] = np.cumsum(counts_h)[:-1]
        seg = np.arange(len(live) + 1, dtype=np.int64)
        # counts and unit offsets staged by nms in its one host->device copy
        r = TMREngine.nms(lg, bx, rf, None, counts_h, unit_off, seg, iou_threshold, want_keep=want_keep)
        for i, g in enumerate(live):
            outs[g] = tuple(x[i] for x in r)
    return outs


def NMS(pred_logits, pred_boxes, ref_points, iou_threshold=0.15):
    """TM_utils.py:307-315: per-image NMS; mutates and returns the lists."""
    outs = _nms_lists(pred_logits, pred_boxes, ref_points, iou_threshold)
    for g in range(len(pred_logits)):
        if g in outs:
            pred_logits[g], pred_boxes[g], ref_points[g] = outs[g]
    return pred_logits, pred_boxes, ref_points


def NMS_process(boxes, logits, iou_threshold=0.65):
    """TM_utils.py:317-323: keep indices (int64, descending-score order)."""
    if boxes.shape[0] == 0:
        return torch.zeros(0, dtype=torch.int64, device=boxes.device)
    refs = torch.zeros((boxes.shape[0], 2), dtype=torch.float32, device=boxes.device)
    outs = _nms_lists([logits], [boxes], [refs], iou_threshold, want_keep=True)
    return outs[0][3]
