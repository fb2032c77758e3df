"""TEST INFRASTRUCTURE ONLY -- generates tests/golden/*.npz from the reference.

Runs the reference's own hot-path code, imported file-by-file from
/root/reference (models/template_matching.py, models/regression_head.py,
models/matching_net.py, models/encoders.py, utils/TM_utils.py), on seeded
small inputs and stores inputs + outputs as .npz fixtures.  Nothing from the
reference is copied into the repo; only data is written.

torchvision is absent from this image, so ``torchvision.ops.roi_align`` and
``torchvision.ops.nms`` are provided by stubs:
  * roi_align -> the C restatement (oracle/tmr_oracle.c); the stub also
    records the roi / output size the reference computed, which pins the
    template sizing arithmetic (template_matching.py:56-75);
  * nms -> an independent pure-Python transcription of torchvision 0.19's
    CPU nms (below), so the NMS fixtures cross-check the C restatement but
    stay UNPINNED against real torchvision.

Usage (in this container only; /root/reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python oracle/make_golden.py
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import types
from types import SimpleNamespace

sys.dont_write_bytecode = True

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import oracle  # noqa: E402

sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

synth = load_package().synth

REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
ROI_LOG = []


# ---------------------------------------------------------------- stubs
def _stub_roi_align(inp, boxes, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=False):
    assert spatial_scale == 1.0 and sampling_ratio == -1 and aligned, "only the path's call form"
    assert inp.shape[0] == 1 and len(boxes) == 1 and boxes[0].shape[0] == 1
    roi = boxes[0][0].detach().cpu().numpy().astype(np.float32)
    ph, pw = output_size
    ROI_LOG.append((roi.copy(), int(ph), int(pw)))
    return torch.from_numpy(oracle.roi_align(inp[0], roi, int(ph), int(pw)))[None]


def py_nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """Independent transcription of torchvision 0.19 csrc/ops/cpu/nms_kernel.cpp."""
    b = boxes.detach().cpu().numpy().astype(np.float32)
    s = scores.detach().cpu().numpy().astype(np.float32)
    n = b.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64)
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    with np.errstate(invalid="ignore", over="ignore"):
        areas = (x2 - x1) * (y2 - y1)
    # scores.sort(stable=true, descending=true): NaN of either sign first (torch
    # orders NaN above +inf), -0.0 == +0.0, ties by index -- np.argsort(-s)
    # would put NaN last
    order = torch.sort(torch.from_numpy(s), stable=True, descending=True).indices.numpy()
    sup = np.zeros(n, bool)
    keep = []
    f = np.float32
    for _i in range(n):
        i = order[_i]
        if sup[i]:
            continue
        keep.append(i)
        for _j in range(_i + 1, n):
            j = order[_j]
            if sup[j]:
                continue
            # Python's max(a, b) / min(a, b) pick like std::max(a, b) / std::min(a, b)
            # (b only when b > a / b < a), NaN included
            xx1 = max(x1[i], x1[j]); yy1 = max(y1[i], y1[j])
            xx2 = min(x2[i], x2[j]); yy2 = min(y2[i], y2[j])
            with np.errstate(invalid="ignore", over="ignore", divide="ignore"):
                w = max(f(0), f(xx2 - xx1)); h = max(f(0), f(yy2 - yy1))
                inter = f(w * h)
                ovr = f(inter / f(f(areas[i] + areas[j]) - inter))
            if float(ovr) > float(iou_threshold):
                sup[j] = True
    return torch.tensor(keep, dtype=torch.int64)


def _install_stubs():
    tv = types.ModuleType("torchvision")
    ops = types.ModuleType("torchvision.ops")
    bx = types.ModuleType("torchvision.ops.boxes")
    ops.roi_align = _stub_roi_align
    ops.nms = py_nms
    bx.box_area = lambda b: (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    tv.ops = ops
    ops.boxes = bx
    sys.modules.update({"torchvision": tv, "torchvision.ops": ops, "torchvision.ops.boxes": bx})


def _pkg(name, path):
    m = types.ModuleType(name)
    m.__path__ = [path]
    sys.modules[name] = m


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


def import_reference():
    """Load the hot-path files, bypassing models/__init__.py (torchvision.models)."""
    _install_stubs()
    _pkg("models", REF + "/models")
    _pkg("models.backbone", REF + "/models/backbone")
    _pkg("models.backbone.sam", REF + "/models/backbone/sam")
    _pkg("utils", REF + "/utils")
    _load("models.backbone.sam.common", REF + "/models/backbone/sam/common.py")
    _load("models.encoders", REF + "/models/encoders.py")
    tm = _load("models.template_matching", REF + "/models/template_matching.py")
    rh = _load("models.regression_head", REF + "/models/regression_head.py")
    mn = _load("models.matching_net", REF + "/models/matching_net.py")
    tu = _load("utils.TM_utils", REF + "/utils/TM_utils.py")
    return SimpleNamespace(tm=tm, rh=rh, mn=mn, tu=tu)


class FakeBackbone(torch.nn.Module):
    """Passthrough encoder: the path starts at the SAM features."""

    def __init__(self, c):
        super().__init__()
        self.num_channels = c

    def forward(self, x):
        return x


def make_args(**kw):
    a = dict(emb_dim=16, fusion=True, ablation_no_box_regression=False, encoder="original",
             feature_upsample=True, no_matcher=False, template_type="roi_align", squeeze=False,
             decoder_num_layer=1, decoder_kernel_size=3, modeltype="matching_net")
    a.update(kw)
    return SimpleNamespace(**a)


# ---------------------------------------------------------------- fixtures
def gen_xcorr(R):
    cases = [(8, 32, 32, k, k, False) for k in (1, 3, 5, 7, 9, 15, 31)]
    cases += [(8, 32, 32, 3, 7, False), (8, 32, 32, 11, 5, False), (64, 16, 16, 5, 5, False),
              (8, 32, 32, 5, 5, True), (16, 24, 40, 9, 3, True)]
    d = {}
    for i, (C, H, W, h, w, sq) in enumerate(cases):
        f = torch.from_numpy(synth.normal(100 + i, (1, C, H, W)))
        t = torch.from_numpy(synth.normal(200 + i, (1, C, h, w)))
        m = R.tm.TemplateMatching("roi_align", squeeze=sq)
        out = m.cross_correlation(f, t)
        d[f"c{i}_meta"] = np.array([C, H, W, h, w, int(sq)], np.int64)
        d[f"c{i}_f"] = f.numpy(); d[f"c{i}_t"] = t.numpy(); d[f"c{i}_out"] = out.numpy()
    d["n"] = np.array(len(cases))
    return d


def gen_template(R):
    H = W = 32
    C = 8
    f = torch.from_numpy(synth.normal(300, (1, C, H, W)))
    boxes = [
        [0.1, 0.2, 0.3, 0.5], [0.0, 0.0, 1.0, 1.0], [-0.2, -0.1, 0.25, 0.3], [0.7, 0.8, 1.3, 1.2],
        [0.5, 0.5, 0.52, 0.53], [0.31, 0.31, 0.3125, 0.3125], [0.25, 0.25, 0.375, 0.375],
        [0.123, 0.456, 0.789, 0.901], [0.0, 0.5, 0.03125, 0.59375], [0.96, 0.96, 1.0, 1.0],
    ]
    for i in range(20):
        u = synth.uniform(400 + i, 4)
        x1, y1 = u[0] * 0.8, u[1] * 0.8
        boxes.append([x1, y1, x1 + 0.02 + u[2] * 0.3, y1 + 0.02 + u[3] * 0.3])
    boxes = np.array(boxes, np.float32)
    m = R.tm.TemplateMatching("roi_align")
    rois, sizes, temps = [], [], []
    for b in boxes:
        ROI_LOG.clear()
        t = m.extract_template(f, torch.from_numpy(b))
        roi, ph, pw = ROI_LOG[0]
        rois.append(roi); sizes.append((ph, pw)); temps.append(t[0].numpy().ravel())
    protos = []
    mp = R.tm.TemplateMatching("prototype")
    for b in boxes:
        protos.append(mp.extract_prototype(f, torch.from_numpy(b)).numpy().ravel())
    return dict(f=f.numpy(), boxes=boxes, rois=np.array(rois), sizes=np.array(sizes, np.int64),
                templates=np.concatenate(temps), protos=np.array(protos))


FORWARD_VARIANTS = {
    "default": {},
    "squeeze": dict(squeeze=True),
    "prototype": dict(template_type="prototype"),
    "nofusion": dict(fusion=False),
    "noboxreg": dict(ablation_no_box_regression=True),
    "twolayer_k5": dict(decoder_num_layer=2, decoder_kernel_size=5),
    "noupsample": dict(feature_upsample=False),
    "nomatcher": dict(no_matcher=True),
}


def gen_forward(R, name, kw, cin=16, emb=16, B=2, h=16, w=16, seed=0):
    args = make_args(emb_dim=emb, **kw)
    torch.manual_seed(seed)
    model = R.mn.matching_net(FakeBackbone(cin), args).eval()
    # reference init leaves every bias at 0; give the heads a non-trivial
    # bias so the fixture also exercises the bias path
    with torch.no_grad():
        model.objectness_head.head[0].bias.fill_(0.25)
        if model.ltrbs_head is not None:
            model.ltrbs_head.head[0].bias.copy_(torch.tensor([0.05, -0.05, 0.1, -0.1]))
        model.matcher is not None and model.matcher.scale.fill_(1.25)
    feats = torch.from_numpy(synth.sam_features(seed + 11, B, cin, h, w))
    Hm = 2 * h if args.feature_upsample else h
    ex, ks = synth.exemplar_set(seed + 12, B, 2, Hm, Hm * w // h, 3, 9)
    exemplars = [torch.from_numpy(ex[b]) for b in range(B)]
    with torch.no_grad():
        os_, bs_, ftm, f0 = model(feats, exemplars)
    d = {f"sd.{k}": v.detach().numpy() for k, v in model.state_dict().items()}
    d.update(feats=feats.numpy(), exemplars=ex, o=os_[0].numpy(), f_tm=ftm[0].numpy(),
             f0=f0.numpy(), args=np.array(json.dumps(vars(args))))
    if bs_[0] is not None:
        d["b"] = bs_[0].numpy()
    return d


def _flatten_lists(prefix, lists):
    d = {}
    counts = np.array([x.shape[0] for x in lists], np.int64)
    d[prefix + "_counts"] = counts
    d[prefix] = np.concatenate([x.numpy() for x in lists]) if len(lists) else np.zeros(0)
    return d


def _crafted_logits(seed, B, H, W):
    """Logit maps with isolated peaks, plateaus, saturation and empty images."""
    o = torch.from_numpy(synth.normal(seed, (B, 1, H, W)) * 2.0 - 1.0)
    o[0, 0, 5:8, 5:8] = 3.0                  # plateau of equal probabilities
    o[0, 0, 10, 3:6] = 40.0                  # sigmoid saturates to exactly 1.0
    o[0, 0, 0, 0] = 6.0                      # corner peak (zero-padded border)
    o[0, 0, H - 1, W - 1] = 6.0
    if B > 1:
        o[1] = -20.0                         # no candidate at all -> dummy row
    if B > 2:
        o[2, 0, ::4, ::4] = 1.5              # lattice of isolated peaks
    return o


def gen_pred_boxes(R):
    B, H, W = 4, 24, 32
    cases = []
    # exemplar sizes chosen to hit all 5 adaptive kernels (TM_utils.py:367-377)
    ex_sizes = {"full": (0.2, 0.25), "center": (1.0 / 48, 1.0 / 64), "vert": (1.0 / 48, 0.1),
                "horz": (0.1, 1.0 / 64), "cross": (2.5 / 24, 2.5 / 32)}
    d = {}
    ci = 0
    for kname, (eh, ew) in ex_sizes.items():
        for thr in (0.1, 0.25, 0.4, 0.7):
            for flags in ((True, False, False), (True, True, False), (True, False, True),
                          (False, False, False)):
                box_reg, ab_b, ab_c = flags
                if kname != "full" and flags != (True, False, False):
                    continue
                o = _crafted_logits(500 + ci, B, H, W)
                reg = torch.from_numpy(synth.normal(600 + ci, (B, 4, H, W)) * 0.3)
                ex = []
                for b in range(B):
                    u = synth.uniform(700 + ci * 8 + b, 2)
                    x1, y1 = float(u[0] * 0.6), float(u[1] * 0.6)
                    ex.append(torch.tensor([[x1, y1, x1 + ew, y1 + eh], [0.1, 0.1, 0.2, 0.2]],
                                           dtype=torch.float32))
                if ci % 7 == 3:  # clamped exemplar coordinates
                    ex[0] = torch.tensor([[-0.1, 0.5, 0.2, 1.3]], dtype=torch.float32)
                batch = {"regression_ablation_b": ab_b, "regression_ablation_c": ab_c}
                L, Bx, Rf = R.tu.Get_pred_boxes([o], [reg] if box_reg else [None], ex, batch,
                                                thr, box_reg)
                probs = np.stack([o[b].sigmoid().squeeze(0).numpy() for b in range(B)])
                d[f"c{ci}_meta"] = np.array(json.dumps(dict(kernel=kname, thr=thr, box_reg=box_reg,
                                                             ab_b=ab_b, ab_c=ab_c)))
                d[f"c{ci}_o"] = o.numpy(); d[f"c{ci}_reg"] = reg.numpy()
                d[f"c{ci}_prob"] = probs
                d[f"c{ci}_ex"] = np.stack([e[0].numpy() for e in ex])
                d.update(_flatten_lists(f"c{ci}_logits", L))
                d.update(_flatten_lists(f"c{ci}_boxes", Bx))
                d.update(_flatten_lists(f"c{ci}_refs", Rf))
                ci += 1
    d["n"] = np.array(ci)
    return d


PRED_BOX_EX_SIZES = {"full": (0.2, 0.25), "center": (1.0 / 48, 1.0 / 64), "vert": (1.0 / 48, 0.1),
                     "horz": (0.1, 1.0 / 64), "cross": (2.5 / 24, 2.5 / 32)}


def _store_pred_boxes(R, d, ci, meta, o, reg, ex, thr, box_reg, ab_b=False, ab_c=False):
    batch = {"regression_ablation_b": ab_b, "regression_ablation_c": ab_c}
    B = o.shape[0]
    L, Bx, Rf = R.tu.Get_pred_boxes([o], [reg] if box_reg else [None], ex, batch, thr, box_reg)
    probs = np.stack([o[b].sigmoid().squeeze(0).numpy() for b in range(B)])
    meta = dict(meta, thr=thr, box_reg=box_reg, ab_b=ab_b, ab_c=ab_c)
    d[f"c{ci}_meta"] = np.array(json.dumps(meta))
    d[f"c{ci}_o"] = o.numpy(); d[f"c{ci}_reg"] = reg.numpy()
    d[f"c{ci}_prob"] = probs
    d[f"c{ci}_ex"] = np.stack([e[0].numpy() for e in ex])
    d.update(_flatten_lists(f"c{ci}_logits", L))
    d.update(_flatten_lists(f"c{ci}_boxes", Bx))
    d.update(_flatten_lists(f"c{ci}_refs", Rf))


def gen_pred_boxes_nonfinite(R):
    """Get_pred_boxes on maps holding NaN / +-inf (TM_utils.py:246-254, 359):
    torch.max over the masked taps propagates NaN, so a pixel with a NaN
    anywhere in its masked window is never a peak.  Per adaptive kernel shape:
    a would-be peak with a NaN at the FIRST masked tap, one with a NaN at the
    LAST masked tap, a NaN centre, a plateau with a NaN beside it, +inf logits
    (p = 1.0, a saturated pair), -inf logits (p = 0), a NaN regression value
    at a peak; then an all-NaN image (dummy row) and a map sprinkled with
    NaN / +-inf."""
    B, H, W = 3, 24, 32
    d = {}
    ci = 0
    for kname, (eh, ew) in PRED_BOX_EX_SIZES.items():
        taps = [(dy, dx) for dy in (-1, 0, 1) for dx in (-1, 0, 1)]
        mask = oracle.adaptive_kernel(np.float32(eh), np.float32(ew), H, W)
        on = [t for t, m in zip(taps, mask.ravel()) if m]
        for thr, box_reg in ((0.1, True), (0.5, True), (0.25, False)):
            o = torch.from_numpy((synth.normal(1500 + ci, (B, 1, H, W)) * 0.5 - 2.0).astype(np.float32))
            reg = torch.from_numpy((synth.normal(1600 + ci, (B, 4, H, W)) * 0.3).astype(np.float32))
            m = o[0, 0]
            nan = float("nan")
            # a would-be peak, NaN at the first masked tap (row-major), and at the last
            m[4, 4] = 3.0; m[4 + on[0][0], 4 + on[0][1]] = nan
            m[4, 12] = 3.0; m[4 + on[-1][0], 12 + on[-1][1]] = nan
            m[4, 20] = 3.0                       # a clean peak for comparison
            m[10, 5] = nan                       # NaN centre
            m[10:12, 12:15] = 2.0; m[10, 15] = nan   # plateau, NaN beside its right end
            m[16, 3] = float("inf"); m[16, 4] = float("inf")   # saturated p = 1.0 pair
            m[16, 10] = float("inf")             # lone +inf
            m[15:18, 19:22] = 1.0; m[16, 20] = float("-inf")   # -inf inside a ring of equal peaks
            m[20, 28] = 2.5                      # a peak whose regression holds NaN
            reg[0, 2, 20, 28] = nan
            m[0, 0] = nan; m[0, 1] = 2.0         # NaN in the zero-padded corner's window
            m[H - 1, W - 1] = 4.0; m[H - 2, W - 2] = nan
            o[1] = nan                           # every pixel NaN: the dummy row
            flat = o[2].view(-1)
            u = synth.uniform(1700 + ci, 3 * 40)
            for j in range(40):
                flat[int(u[3 * j] * flat.numel()) % flat.numel()] = [nan, float("inf"), float("-inf")][
                    int(u[3 * j + 1] * 3) % 3]
                flat[int(u[3 * j + 2] * flat.numel()) % flat.numel()] = 1.5
            ex = []
            for b in range(B):
                x1, y1 = 0.1 + 0.05 * b, 0.2
                ex.append(torch.tensor([[x1, y1, x1 + ew, y1 + eh]], dtype=torch.float32))
            _store_pred_boxes(R, d, ci, dict(kernel=kname), o, reg, ex, thr, box_reg)
            ci += 1
    d["n"] = np.array(ci)
    return d


def gen_nms_nonfinite(R):
    """NMS with non-finite inputs (TM_utils.py:307-323 -> torchvision nms):
    NaN scores of both signs sort first (torch.sort descending), +-inf
    scores, -0.0 / +0.0 ties, NaN / inf box coordinates (a NaN area gives a
    NaN IoU: never suppresses, never suppressed); small sets (one-workgroup
    path) and sets over 256 rows (the binned path)."""
    d = {}
    cases = []
    qn = np.array([0xffc00000], np.uint32).view(np.float32)[0]   # x86's default NaN (negative)
    b = np.array([[0, 0, 1, 1], [0.1, 0, 1.1, 1], [0, 0.1, 1, 1.1], [0.05, 0.05, 1, 1],
                  [2, 2, 3, 3], [2.1, 2, 3.1, 3], [0, 0, 1, 1], [5, 5, 6, 6]], np.float32)
    s = np.array([0.5, np.nan, 0.9, np.inf, 0.0, -0.0, qn, -np.inf], np.float32)
    cases += [(b, s, 0.5), (b, s, 0.15), (b, s, -0.1)]
    s2 = np.array([-0.0, 0.0, -0.0, 0.0, 0.7, 0.7, np.nan, np.nan], np.float32)
    cases.append((b, s2, 0.3))
    b3 = b.copy(); b3[1, 0] = np.nan; b3[3, 2] = np.inf; b3[5] = [np.inf, np.inf, np.inf, np.inf]
    b3[4, 1] = -np.inf
    s3 = np.array([0.9, 0.95, 0.8, 0.85, 0.6, 0.6, 0.5, 0.4], np.float32)
    cases += [(b3, s3, 0.5), (b3, s, 0.15)]
    for i, n in enumerate((40, 300, 700)):
        u = synth.uniform(1900 + i, 6 * n).reshape(n, 6).astype(np.float32)
        xy = u[:, :2] * 0.6
        bx = np.concatenate([xy, xy + 0.05 + u[:, 2:4] * 0.2], 1).astype(np.float32)
        sc = (np.round(u[:, 4] * 8) / 8).astype(np.float32)
        pick = u[:, 5]
        sc[pick < 0.05] = np.nan
        sc[(pick >= 0.05) & (pick < 0.08)] = qn
        sc[(pick >= 0.08) & (pick < 0.1)] = np.inf
        sc[(pick >= 0.1) & (pick < 0.12)] = -np.inf
        sc[(pick >= 0.12) & (pick < 0.15)] = -0.0
        bx[(pick >= 0.15) & (pick < 0.17), 2] = np.nan
        bx[(pick >= 0.17) & (pick < 0.18), 3] = np.inf
        cases.append((bx, sc, [0.5, 0.15, 0.65][i]))
    for i, (bx, sc, thr) in enumerate(cases):
        logits = [torch.from_numpy(np.stack([sc, np.zeros_like(sc)], 1))]
        boxes = [torch.from_numpy(bx.copy())]
        refs = [torch.from_numpy(bx[:, :2].copy())]
        L, Bx, Rf = R.tu.NMS(logits, boxes, refs, thr)
        keep = py_nms(torch.from_numpy(bx), torch.from_numpy(sc), thr).numpy()
        d[f"c{i}_boxes"] = bx; d[f"c{i}_scores"] = sc; d[f"c{i}_thr"] = np.array(thr)
        d[f"c{i}_keep"] = keep; d[f"c{i}_kept_boxes"] = Bx[0].numpy()
        d[f"c{i}_kept_logits"] = L[0].numpy()
    d["n"] = np.array(len(cases))
    return d


def gen_nms(R):
    d = {}
    cases = []
    # ties, duplicates, IoU exactly at threshold, dummy rows, empty
    b = np.array([[0, 0, 1, 1], [0, 0, 1, 1], [0.5, 0, 1.5, 1], [0, 0, 1, 1], [2, 2, 3, 3],
                  [0, 0, 1e-14, 1e-14], [0, 0, 1e-14, 1e-14]], np.float32)
    s = np.array([0.9, 0.9, 0.8, 0.7, 0.7, 0.0, 0.0], np.float32)
    cases.append((b, s, 0.5)); cases.append((b, s, 1.0 / 3.0)); cases.append((b, s, 0.15))
    for i in range(12):
        n = [5, 40, 200, 800][i % 4]
        u = synth.uniform(900 + i, 5 * n).reshape(n, 5).astype(np.float32)
        xy = u[:, :2] * 0.8
        wh = 0.02 + u[:, 2:4] * 0.15
        bx = np.concatenate([xy, xy + wh], 1).astype(np.float32)
        sc = np.round(u[:, 4] * 16) / 16  # many ties
        cases.append((bx, sc.astype(np.float32), [0.15, 0.5, 0.65][i % 3]))
    cases.append((np.zeros((0, 4), np.float32), np.zeros(0, np.float32), 0.5))
    for i, (bx, sc, thr) in enumerate(cases):
        logits = [torch.from_numpy(np.stack([sc, np.zeros_like(sc)], 1))]
        boxes = [torch.from_numpy(bx)]
        refs = [torch.from_numpy(bx[:, :2].copy())]
        if bx.shape[0]:
            L, Bx, Rf = R.tu.NMS(logits, boxes, refs, thr)
            keep = py_nms(torch.from_numpy(bx), torch.from_numpy(sc), thr).numpy()
        else:
            keep = np.zeros(0, np.int64); L, Bx = logits, boxes
        d[f"c{i}_boxes"] = bx; d[f"c{i}_scores"] = sc; d[f"c{i}_thr"] = np.array(thr)
        d[f"c{i}_keep"] = keep; d[f"c{i}_kept_boxes"] = Bx[0].numpy()
    d["n"] = np.array(len(cases))
    return d


def gen_caller(R):
    """demo.Inference.infer / Matching_Trainer.each_step_multi_exemplars call
    sequence (demo.py:106-130, trainer.py:95-118): one forward per exemplar,
    Get_pred_boxes, concat over exemplars, one NMS."""
    cin, emb, h, w, E = 16, 16, 16, 16, 3
    args = make_args(emb_dim=emb)
    torch.manual_seed(3)
    model = R.mn.matching_net(FakeBackbone(cin), args).eval()
    with torch.no_grad():
        model.objectness_head.head[0].bias.fill_(0.5)
    feats = torch.from_numpy(synth.sam_features(31, 1, cin, h, w))
    ex, _ = synth.exemplar_set(32, 1, E, 2 * h, 2 * w, 3, 7)
    d = {f"sd.{k}": v.detach().numpy() for k, v in model.state_dict().items()}
    d.update(feats=feats.numpy(), exemplars=ex)
    for thr, iou in ((0.1, 0.5), (0.5, 0.15), (0.7, 0.5)):
        logits, boxes, refs = [], [], []
        for e in range(E):
            exemplar = [torch.from_numpy(ex[0, e:e + 1])]
            with torch.no_grad():
                o, b, _, _ = model(feats, exemplar)
            batch = {"regression_ablation_b": False, "regression_ablation_c": False}
            L, Bx, Rf = R.tu.Get_pred_boxes(o, b, exemplar, batch, thr, True)
            logits.append(L[0]); boxes.append(Bx[0]); refs.append(Rf[0])
        L, Bx, Rf = R.tu.NMS([torch.cat(logits)], [torch.cat(boxes)], [torch.cat(refs)], iou)
        tag = f"t{int(thr * 100)}_i{int(iou * 100)}"
        d[f"{tag}_logits"] = L[0].numpy(); d[f"{tag}_boxes"] = Bx[0].numpy()
        d[f"{tag}_refs"] = Rf[0].numpy()
        d[f"{tag}_precount"] = np.array(sum(x.shape[0] for x in logits))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--only", nargs="*", help="regenerate only these fixtures (names without .npz)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    torch.set_num_threads(8)
    R = import_reference()
    meta = dict(torch=torch.__version__, threads=torch.get_num_threads(), numpy=np.__version__,
                reference="/root/reference @ 2026-01-16", generator="oracle/make_golden.py",
                stubs="roi_align=oracle C restatement (unpinned); nms=py_nms transcription (unpinned)")
    jobs = {"xcorr": lambda: gen_xcorr(R), "template": lambda: gen_template(R),
            "pred_boxes": lambda: gen_pred_boxes(R), "nms": lambda: gen_nms(R),
            "caller": lambda: gen_caller(R),
            "pred_boxes_nonfinite": lambda: gen_pred_boxes_nonfinite(R),
            "nms_nonfinite": lambda: gen_nms_nonfinite(R)}
    for name, kw in FORWARD_VARIANTS.items():
        jobs[f"forward_{name}"] = (lambda kw=kw, name=name: gen_forward(R, name, kw))
    for name, fn in jobs.items():
        if a.only and name not in a.only:
            continue
        d = fn()
        d["meta"] = np.array(json.dumps(meta))
        np.savez_compressed(os.path.join(a.out, f"{name}.npz"), **d)
        print("wrote", name)


if __name__ == "__main__":
    main()
