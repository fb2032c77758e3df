"""Host-side descriptors for the HIP kernels.

The reference sizes templates and peak kernels with Python scalar math on 0-d
fp32 tensors (models/template_matching.py:56-73, utils/TM_utils.py:236-252,
363-377).  These helpers reproduce that arithmetic exactly in numpy fp32 and
pack it into the tmr_unit_t / tmr_peak_param_t structs of include/tmr.h.
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

import numpy as np

from ._lib import PEAK_DTYPE, TEMPLATE_PROTOTYPE, TEMPLATE_ROI_ALIGN, UNIT_DTYPE

f32 = np.float32

TEMPLATE_TYPES = {"roi_align": TEMPLATE_ROI_ALIGN, "prototype": TEMPLATE_PROTOTYPE}


def clamp01(v) -> np.float32:
    """min(1., max(0., v)) with Python's min/max semantics
    (template_matching.py:58-59, TM_utils.py:237-238)."""
    v = f32(v)
    m = v if v > f32(0.0) else f32(0.0)
    return m if m < f32(1.0) else f32(1.0)


def clamp_box(box) -> np.ndarray:
    b = np.asarray(box, dtype=np.float32).reshape(4)
    return np.array([clamp01(x) for x in b], np.float32)


_F0, _F1 = f32(0.0), f32(1.0)


def _clamp01_fast(v: np.float32) -> np.float32:
    """clamp01 of an fp32 scalar (no conversions: the per-unit path)."""
    m = v if v > _F0 else _F0
    return m if m < _F1 else _F1


def clamp01_vec(v: np.ndarray) -> np.ndarray:
    """clamp01 elementwise with the same semantics (NaN -> 0, like Python's
    `v if v > 0 else 0`), fp32."""
    v = np.asarray(v, np.float32)
    m = np.where(v > f32(0.0), v, f32(0.0)).astype(np.float32)
    return np.where(m < f32(1.0), m, f32(1.0)).astype(np.float32)


def template_sizes(boxes: np.ndarray, H: int, W: int):
    """template_size over [U,4] boxes at once, the same fp32 operations per
    element: (rois [U,4] fp32, ht [U] int, wt [U] int); raises like
    template_size for the first box the reference would reject."""
    c = clamp01_vec(np.asarray(boxes, np.float32).reshape(-1, 4))
    x1, x2 = (c[:, 0] * f32(W)).astype(np.float32), (c[:, 2] * f32(W)).astype(np.float32)
    y1, y2 = (c[:, 1] * f32(H)).astype(np.float32), (c[:, 3] * f32(H)).astype(np.float32)
    wt = np.ceil(x2).astype(np.int64) - np.floor(x1).astype(np.int64)
    ht = np.ceil(y2).astype(np.int64) - np.floor(y1).astype(np.int64)
    wt -= (wt % 2 == 0)
    ht -= (ht % 2 == 0)
    bad = (ht <= 0) | (wt <= 0) | (ht > H) | (wt > W)
    if bad.any():
        template_size(np.asarray(boxes, np.float32).reshape(-1, 4)[int(np.argmax(bad))], H, W)  # raises
    return np.stack([x1, y1, x2, y2], 1).astype(np.float32), ht, wt


def tsplit_windows_vec(ht: np.ndarray, wt: np.ndarray) -> np.ndarray:
    """tsplit_windows over arrays of template sizes."""
    h, w = np.asarray(ht, np.int64), np.asarray(wt, np.int64)
    s = (-(w // 2)) % 8
    return ((h + 4) // 4) * ((w + s + 14) // 8)


def template_size(box, H: int, W: int) -> Tuple[np.ndarray, int, int]:
    """(roi in feature px, Ht, Wt) exactly as extract_template computes them
    (template_matching.py:56-73).  Raises ValueError where the reference would
    ask roi_align for a non-positive output size."""
    b = box if isinstance(box, np.ndarray) and box.dtype == np.float32 and box.shape == (4,) else \
        np.asarray(box, dtype=np.float32).reshape(4)
    c0, c1, c2, c3 = (_clamp01_fast(v) for v in b)
    fW, fH = f32(W), f32(H)
    x1, x2 = c0 * fW, c2 * fW  # fp32 scalar products (np.float32 * np.float32)
    y1, y2 = c1 * fH, c3 * fH
    wt = math.ceil(float(x2)) - math.floor(float(x1))
    ht = math.ceil(float(y2)) - math.floor(float(y1))
    if wt % 2 == 0:
        wt -= 1
    if ht % 2 == 0:
        ht -= 1
    if ht <= 0 or wt <= 0:
        raise ValueError(f"exemplar box {np.asarray(box).tolist()} gives a {ht}x{wt} template "
                         "(the reference's roi_align call fails for it too)")
    if ht > H or wt > W:
        raise ValueError(f"template {ht}x{wt} larger than the {H}x{W} feature map")
    return np.array([x1, y1, x2, y2], np.float32), ht, wt


def prototype_box(box, H: int, W: int) -> np.ndarray:
    """Integer-snapped box of extract_prototype (template_matching.py:44-50)."""
    c = clamp_box(box)
    x1, x2 = f32(c[0] * f32(W)), f32(c[2] * f32(W))
    y1, y2 = f32(c[1] * f32(H)), f32(c[3] * f32(H))
    b = np.array([math.floor(float(x1)), math.floor(float(y1)), math.ceil(float(x2)),
                  math.ceil(float(y2))], np.int32)
    if b[2] <= b[0] or b[3] <= b[1]:
        raise ValueError(f"exemplar box {np.asarray(box).tolist()} selects an empty region")
    return b


def tsplit_windows(ht: int, wt: int) -> int:
    """A-fragment windows per (unit, channel) of the MFMA correlation
    (include/tmr.h, tmr_template_split; csrc/xcorr.hip win_count): windows of
    4 input rows x 8 input columns over the 2 x 8 output patch's input region,
    ceil((h + 1) / 4) * ceil((w + 7 + s) / 8) with s = (-(w // 2)) mod 8
    aligning each window's first column to 8 elements (16 B)."""
    h, w = int(ht), int(wt)
    s = (-(w // 2)) % 8
    return ((h + 4) // 4) * ((w + s + 14) // 8)


def tsplit_rows(units: np.ndarray) -> int:
    """total_rows of tmr_template_split: the sum of tsplit_windows over the units."""
    return int(sum(tsplit_windows(h, w) for h, w in zip(units["ht"], units["wt"])))


SMALL_UNITS = 8  # up to this many units build_units runs per unit


def build_units(boxes: np.ndarray, images: Sequence[int], H: int, W: int, C: int,
                template_type: str = "roi_align"):
    """tmr_unit_t array for U units.  Returns (units, template_floats, max_ht, max_wt)."""
    boxes = np.asarray(boxes, np.float32).reshape(-1, 4)
    U = boxes.shape[0]
    ttype = TEMPLATE_TYPES[template_type]
    units = np.zeros(U, UNIT_DTYPE)
    if ttype == TEMPLATE_ROI_ALIGN and U > SMALL_UNITS:
        # vectorised: the same fp32 arithmetic per unit as template_size
        rois, ht, wt = template_sizes(boxes, H, W)
        units["image"] = np.asarray(images, np.int64)[:U]
        units["type"] = ttype
        units["roi"] = rois
        units["ht"], units["wt"] = ht, wt
        sizes = C * ht * wt
        units["tmpl_offset"] = np.concatenate([[0], np.cumsum(sizes)[:-1]])
        rows = tsplit_windows_vec(ht, wt)
        units["row_offset"] = np.concatenate([[0], np.cumsum(rows)[:-1]])
        return units, int(sizes.sum()), max(1, int(ht.max())), max(1, int(wt.max()))
    # per unit (prototype templates, and few units: the module API's one
    # exemplar per call, where the vector form's per-call overhead dominates)
    off = rows = 0
    max_ht = max_wt = 1
    zero4 = (0, 0, 0, 0)
    for u in range(U):
        if ttype == TEMPLATE_ROI_ALIGN:
            roi, ht, wt = template_size(boxes[u], H, W)
            roi, pbox = tuple(roi.tolist()), zero4
        else:
            pbox = tuple(prototype_box(boxes[u], H, W).tolist())
            roi, ht, wt = (0.0, 0.0, 0.0, 0.0), 1, 1
        units[u] = (int(images[u]), ttype, ht, wt, roi, pbox, off, rows, 0)
        off += C * ht * wt
        rows += tsplit_windows(ht, wt)
        max_ht, max_wt = max(max_ht, ht), max(max_wt, wt)
    return units, off, max_ht, max_wt


def image_ranges(unit_image: Sequence[int], B: int) -> np.ndarray:
    """[B+1] int32 unit ranges per image; units must be sorted by image."""
    if len(unit_image) <= SMALL_UNITS:  # per unit (the module API's calls)
        r, prev = [0] * (B + 1), 0
        for i in unit_image:
            i = int(i)
            if i < prev or i < 0 or i >= B:
                raise ValueError("units must be sorted by image and index images of the batch")
            prev = i
            r[i + 1] += 1
        for b in range(B):
            r[b + 1] += r[b]
        return np.array(r, np.int32)
    ui = np.asarray(unit_image, np.int64)
    if len(ui) and (np.any(np.diff(ui) < 0) or ui.min() < 0 or ui.max() >= B):
        raise ValueError("units must be sorted by image and index images of the batch")
    r = np.zeros(B + 1, np.int32)
    r[1:] = np.cumsum(np.bincount(ui, minlength=B))
    return r


# adaptive_kernel_generater (TM_utils.py:363-377) as 9-bit masks, bit (dy+1)*3+(dx+1)
KERNEL_FULL = 0b111111111
KERNEL_CENTER = 1 << 4
KERNEL_VERT = (1 << 1) | (1 << 4) | (1 << 7)
KERNEL_HORZ = (1 << 3) | (1 << 4) | (1 << 5)
KERNEL_CROSS = KERNEL_VERT | KERNEL_HORZ


def adaptive_mask(ex_h, ex_w, H: int, W: int) -> int:
    """ex_h/ex_w are fp32 (0-d tensor arithmetic); torch compares them with the
    Python double k/H cast to fp32."""
    ex_h, ex_w = f32(ex_h), f32(ex_w)
    nh, nw = 1.0 / H, 1.0 / W
    h3, w3, h2, w2 = f32(nh * 3), f32(nw * 3), f32(nh * 2), f32(nw * 2)
    if ex_h >= h3 and ex_w >= w3:
        return KERNEL_FULL
    if ex_h < h2 and ex_w < w2:
        return KERNEL_CENTER
    if ex_h < h2 and ex_w >= w2:
        return KERNEL_VERT
    if ex_h >= h2 and ex_w < w2:
        return KERNEL_HORZ
    return KERNEL_CROSS


def mask_to_kernel(mask: int):
    """9-bit mask -> the 3x3 list adaptive_kernel_generater returns."""
    return [[(mask >> (r * 3 + c)) & 1 for c in range(3)] for r in range(3)]


def peak_params(boxes: np.ndarray, H: int, W: int, cls_ths: float, box_reg: bool = True,
                ablation_b: bool = False, ablation_c: bool = False) -> np.ndarray:
    """tmr_peak_param_t per unit (TM_utils.py:236-252, 264-276)."""
    boxes = np.asarray(boxes, np.float32).reshape(-1, 4)
    P = np.zeros(boxes.shape[0], PEAK_DTYPE)
    thr = f32(cls_ths)
    mode = 2 if not box_reg else (1 if ablation_c else 0)
    # vectorised: the same fp32 arithmetic per unit as adaptive_mask
    c = clamp01_vec(boxes)
    bw = (c[:, 2] - c[:, 0]).astype(np.float32)
    bh = (c[:, 3] - c[:, 1]).astype(np.float32)
    nh, nw = 1.0 / H, 1.0 / W
    h3, w3, h2, w2 = f32(nh * 3), f32(nw * 3), f32(nh * 2), f32(nw * 2)
    mask = np.select([(bh >= h3) & (bw >= w3), (bh < h2) & (bw < w2), (bh < h2) & (bw >= w2),
                      (bh >= h2) & (bw < w2)],
                     [KERNEL_FULL, KERNEL_CENTER, KERNEL_VERT, KERNEL_HORZ], KERNEL_CROSS)
    P["thr"] = thr
    P["scale_w"] = f32(1.0) if ablation_b else bw
    P["scale_h"] = f32(1.0) if ablation_b else bh
    P["mask"] = mask
    P["mode"] = mode
    return P


def nms_offsets(counts: np.ndarray, seg_units: np.ndarray):
    """Per-image candidate-union sizes (dummy row for an empty unit,
    TM_utils.py:288-291) -> (cand_off[G+1], nb_off[G+1], max_cand): nb_off
    are the prefix sums of ceil(n_g / 64), the 64-row blocks of tmr_nms."""
    counts = np.asarray(counts, np.int64)
    G = len(seg_units) - 1
    n = np.zeros(G, np.int64)
    for g in range(G):
        c = counts[seg_units[g]:seg_units[g + 1]]
        n[g] = int(np.maximum(c, 1).sum())
    cand_off = np.zeros(G + 1, np.int64)
    cand_off[1:] = np.cumsum(n)
    nb_off = np.zeros(G + 1, np.int64)
    nb_off[1:] = np.cumsum((n + 63) // 64)
    return cand_off, nb_off, int(n.max()) if G else 0
