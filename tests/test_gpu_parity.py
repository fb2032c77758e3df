"""GPU parity: libtmr.so (through the C ABI via the tmr_amd modules) against
the golden vectors from the reference and the CPU oracle.

Tolerances (written here):
  fp32 maps (xcorr, decoder/heads, o/b): normwise max|d|/max|ref| <= 1e-5
  templates (RoIAlign), upsample, peaks, keep indices, counts: bit-exact
  box corners: bit-exact vs the oracle and vs the reference's own outputs
  (the decode's exp restated through the reference-exp table, exp_table.py)
"""
import json
import os

import numpy as np
import pytest
import torch

import oracle
import tmr_amd
from tmr_amd import host, synth

pytestmark = pytest.mark.gpu

TOL = 1e-5
DEV = torch.device("cuda:0")


def normwise(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def corner_ok(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    if a.size == 0:
        return True
    scale = np.spacing(np.abs(b).max(axis=-1, keepdims=True).astype(np.float32))
    return bool((np.abs(a.astype(np.float64) - b) <= 2 * scale).all())


def cuda(x):
    return torch.as_tensor(x).to(DEV)


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def bits_equal_nan(a, b):
    """bits_equal, except that a NaN matches any NaN (the payload of a NaN
    that propagates through exp / products is not part of the contract)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    if a.shape != b.shape or not np.array_equal(np.isnan(a), np.isnan(b)):
        return False
    m = ~np.isnan(b)
    return np.array_equal(a[m].view(np.uint32), b[m].view(np.uint32))


# ----------------------------------------------------------------- templates
def test_roi_align_bitexact_vs_oracle(golden):
    g = golden("template")
    f = cuda(g["f"])
    m = tmr_amd.TemplateMatching("roi_align").to(DEV)
    mp = tmr_amd.TemplateMatching("prototype").to(DEV)
    off = 0
    for i, box in enumerate(g["boxes"]):
        t = m.extract_template(f, torch.from_numpy(box)).cpu().numpy()[0]
        ht, wt = g["sizes"][i]
        assert t.shape == (f.shape[1], ht, wt)
        ref = g["templates"][off:off + t.size].reshape(t.shape)
        off += t.size
        assert bits_equal(t, ref), i
        p = mp.extract_prototype(f, torch.from_numpy(box)).cpu().numpy().ravel()
        assert normwise(p, g["protos"][i]) <= TOL


@pytest.mark.parametrize("C,H,W", [(64, 128, 128), (32, 96, 96)])
def test_roi_align_bitexact_large(C, H, W):
    f = synth.normal(3, (1, C, H, W))
    boxes = []
    for k in (1, 3, 7, 15, 31):
        boxes.append(synth.exemplar_box(k, H, W, 5, 9))
    boxes.append(np.array([0.1, 0.2, 0.9, 0.95], np.float32))  # big template, sampling grid > 1
    boxes.append(np.array([-0.2, 0.5, 0.3, 1.4], np.float32))  # clamped
    m = tmr_amd.TemplateMatching("roi_align").to(DEV)
    fd = cuda(f)
    for box in boxes:
        roi, ht, wt = oracle.template_size(box, H, W)
        ref = oracle.roi_align(f[0], roi, ht, wt)
        got = m.extract_template(fd, torch.from_numpy(box)).cpu().numpy()[0]
        assert bits_equal(got, ref)


# ----------------------------------------------------------------- xcorr
def test_xcorr_golden(golden):
    g = golden("xcorr")
    for i in range(int(g["n"])):
        C, H, W, h, w, sq = g[f"c{i}_meta"].tolist()
        f, t, ref = g[f"c{i}_f"], g[f"c{i}_t"], g[f"c{i}_out"]
        # drive tmr_xcorr directly with the golden template (no RoIAlign)
        units = np.zeros(1, tmr_amd._lib.UNIT_DTYPE)
        units["ht"], units["wt"], units["tmpl_offset"] = h, w, 0
        from tmr_amd._lib import PREC_CODES, XCORR_ALGOS, ptr, stream, xcorr
        from tmr_amd.engine import _units_to_device
        fd, td = cuda(f), cuda(t.reshape(-1))
        out = torch.empty((1, 1 if sq else C, H, W), device=DEV)
        relu = torch.empty_like(out)
        work = torch.empty((1, C, H, W), device=DEV) if sq else None
        scale = torch.ones(1, device=DEV)
        ud = _units_to_device(units, DEV)
        iu = cuda(np.array([0, 1], np.int32))
        amax = torch.zeros(1, device=DEV)  # per-unit max |f_TM| (one unit)
        xcorr(f=ptr(fd), templates=ptr(td), units=ptr(ud), img_units=ptr(iu), scale=ptr(scale), out=ptr(out),
              relu_out=ptr(relu), work=ptr(work), out_absmax=ptr(amax), B=1, C=C, H=H, W=W, U=1, max_ht=h,
              max_wt=w, squeeze=sq, algo=XCORR_ALGOS["valu"], min_k=1, prec=PREC_CODES["fp32"], stream=stream())
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert normwise(got, ref) <= TOL, (i, normwise(got, ref))
        assert amax.item() == np.abs(got).max()  # fused |f_TM| max (split decoder scale)
        assert np.array_equal(relu.cpu().numpy(), np.maximum(got, 0))
        # the pad border is exactly zero
        if h > 1:
            assert (got[..., : h // 2, :] == 0).all() and (got[..., H - h // 2:, :] == 0).all()


@pytest.mark.parametrize("k", [3, 9, 15, 31])
def test_xcorr_large_vs_oracle(k):
    C, H, W = 16, 128, 128
    f = synth.normal(10 + k, (2, C, H, W))
    boxes = np.stack([synth.exemplar_box(k, H, W, 3, 11), synth.exemplar_box(k, H, W, 40, 2)])
    m = tmr_amd.TemplateMatching("roi_align").to(DEV)
    with torch.no_grad():
        m.scale.fill_(0.75)
    got = m(cuda(f), [torch.from_numpy(b[None]) for b in boxes]).cpu().numpy()
    for b in range(2):
        roi, ht, wt = oracle.template_size(boxes[b], H, W)
        t = oracle.roi_align(f[b], roi, ht, wt)
        ref = oracle.xcorr(f[b], t, 0.75)
        assert normwise(got[b], ref) <= TOL


@pytest.mark.parametrize("H,W", [(29, 37), (40, 30), (33, 64), (70, 128)])
def test_xcorr_units_both_kernels_vs_oracle(H, W):
    """Several units per image with mixed (rectangular) template sizes through
    TMREngine.match: W % 4 == 0 runs xcorr_rows_kernel (lane tiles over the
    whole band, border computed in-tile), other widths the generic
    xcorr_kernel; band edges (H not a multiple of the 32-row band) included."""
    C = 24
    P = {k: v.to(DEV) for k, v in synth.reference_state_dict(0, cin=16, emb=C).items()}
    eng = tmr_amd.TMREngine(P, tmr_amd.PathConfig(emb_dim=C))
    fp = synth.normal(77 + W, (2, C, H, W))
    shapes = [(3, 3), (7, 5), (13, 9), (1, 1), (5, 11), (9, 3)]
    boxes, ui = [], []
    for u, (kh, kw) in enumerate(shapes):
        kh, kw = min(kh, H // 2 * 2 - 1), min(kw, W // 2 * 2 - 1)
        boxes.append(synth.exemplar_box(kh, H, W, (5 * u) % (H - kh), (7 * u) % (W - kw), kw))
        ui.append(u // 3)
    boxes = np.stack(boxes)
    got, _ = eng.match(cuda(fp), ui, boxes)
    got = got.cpu().numpy()
    for u in range(len(ui)):
        roi, ht, wt = oracle.template_size(boxes[u], H, W)
        t = oracle.roi_align(fp[ui[u]], roi, ht, wt)
        ref = oracle.xcorr(fp[ui[u]], t, 1.0)
        assert normwise(got[u], ref) <= TOL, (u, ht, wt, normwise(got[u], ref))
        ph, pw = ht // 2, wt // 2
        if ph:
            assert (got[u][:, :ph] == 0).all() and (got[u][:, H - ph:] == 0).all()
        if pw:
            assert (got[u][:, :, :pw] == 0).all() and (got[u][:, :, W - pw:] == 0).all()


# ----------------------------------------------------------------- convs
@pytest.mark.parametrize("C,N,H,W,ks", [(64, 64, 32, 40, 3), (40, 72, 17, 33, 3), (16, 16, 24, 24, 5),
                                        (24, 8, 20, 20, 1), (1024, 1024, 16, 32, 3), (12, 12, 9, 9, 7)])
def test_decoder_conv_vs_torch(C, N, H, W, ks):
    torch.manual_seed(C + N + ks)
    x = torch.randn(2, C, H, W)
    dec = tmr_amd.Decoder_model(C, 1, ks)
    if N != C:
        dec.layer[0] = torch.nn.Conv2d(C, N, ks, padding=ks // 2)
    with torch.no_grad():
        dec.layer[0].bias.normal_()
    ref = torch.nn.functional.leaky_relu(dec.layer[0](x), 0.01).detach().numpy()
    got = dec.to(DEV)(x.to(DEV)).cpu().numpy()
    assert normwise(got, ref) <= TOL


SPLIT_TOL = {"fp32": TOL, "f16": 1e-3, "bf16": 1e-2}


@pytest.mark.parametrize("prec", ["fp32", "bf16", "f16"])
@pytest.mark.parametrize("C,N,H,W,ks,leaky", [(64, 64, 32, 40, 3, True), (40, 72, 17, 33, 3, True),
                                              (13, 200, 9, 70, 3, False), (1024, 256, 16, 32, 3, True),
                                              (16, 16, 24, 24, 5, True), (24, 8, 20, 20, 1, False),
                                              (12, 12, 9, 9, 7, True), (512, 2048, 16, 16, 3, True)])
def test_split_conv_vs_torch(C, N, H, W, ks, leaky, prec):
    """Split 16-bit MFMA kernel (tmr_split_conv) vs ATen conv2d (fp32
    CPU) with an acc_init input: "fp32" (3-term fp16 split) within the 1e-5
    contract, one-term bf16 / f16 within their stated tolerances."""
    from tmr_amd._lib import PREC_CODES, call, ptr, stream
    from tmr_amd.engine import absmax, pack_split_w, pack_split_x
    torch.manual_seed(C * 7 + N + ks)
    x = torch.randn(2, C, H, W)
    w = torch.randn(N, C, ks, ks) * (1.0 / (ks * C ** 0.5))
    b = torch.randn(N)
    init = torch.randn(2, N, H, W)
    ref = torch.nn.functional.conv2d(x, w, b, padding=ks // 2) + init
    if leaky:
        ref = torch.nn.functional.leaky_relu(ref, 0.01)
    xd, wd, bd, initd = cuda(x), cuda(w), cuda(b), cuda(init)
    wp, wmax = pack_split_w(wd, C, prec)
    xmax = absmax(xd)
    xp = pack_split_x(xd, ks, prec, xmax)
    out = torch.empty((2, N, H, W), device=DEV)
    call("tmr_split_conv", ptr(xp), C, None, None, 0, 2, H, W, ks, PREC_CODES[prec], ptr(wp),
         ptr(wmax), ptr(xmax), ptr(bd), N, int(leaky), None, ptr(initd), ptr(out), 0, stream())
    torch.cuda.synchronize()
    assert normwise(out.cpu().numpy(), ref.numpy()) <= SPLIT_TOL[prec]


@pytest.mark.parametrize("scale", [1e-6, 1.0, 3e5])
def test_split_conv_scales_and_two_sources(scale):
    """Activations far from unit scale (the power-of-two split scale), zero
    rows, and the two-source virtual concat (src0 per image via unit_image,
    src1 per unit) of tmr_split_conv (heads) vs the unsplit fp32 reference."""
    from tmr_amd._lib import call, ptr, stream
    from tmr_amd.engine import absmax, pack_split_w, pack_split_x
    torch.manual_seed(3)
    B, U, C0, C1, N, H, W = 2, 3, 24, 40, 136, 18, 35
    x0 = torch.randn(B, C0, H, W) * scale
    x1 = torch.randn(U, C1, H, W) * scale
    x1[1] = 0.0
    ui = np.array([1, 0, 1], np.int32)
    w = torch.randn(N, C0 + C1, 3, 3) * 0.01
    bias = torch.randn(N) * scale * 0.01
    hw = torch.zeros(((N + 127) // 128) * 128, 5)
    hw[:N] = torch.randn(N, 5)
    xcat = torch.cat([x0[torch.from_numpy(ui).long()], x1], 1)
    act = torch.nn.functional.leaky_relu(torch.nn.functional.conv2d(xcat.double(), w.double(),
                                                                    bias.double(), padding=1), 0.01)
    ref = torch.einsum("unhw,nj->ujhw", act, hw[:N].double()).numpy()
    d = {k: cuda(v) for k, v in dict(x0=x0, x1=x1, w=w, b=bias, hw=hw).items()}
    uid = cuda(torch.from_numpy(ui))
    wp, wmax = pack_split_w(d["w"], C0, "fp32")
    xmax = absmax(d["x1"], absmax(d["x0"]))
    xp0 = pack_split_x(d["x0"], 3, "fp32", xmax)
    xp1 = pack_split_x(d["x1"], 3, "fp32", xmax)
    part = torch.empty(tmr_amd._lib.size("heads_partials", N, U, H, W), device=DEV)
    call("tmr_split_conv", ptr(xp0), C0, ptr(uid), ptr(xp1), C1, U, H, W, 3, 0, ptr(wp),
         ptr(wmax), ptr(xmax), ptr(d["b"]), N, 1, ptr(d["hw"]), None, ptr(part), 0, stream())
    o = torch.empty((U, 1, H, W), device=DEV)
    bb = torch.empty((U, 4, H, W), device=DEV)
    hb = torch.zeros(5, device=DEV)
    call("tmr_heads_reduce", ptr(part), N, 128, U, H, W, ptr(hb), ptr(o), ptr(bb), stream())
    torch.cuda.synchronize()
    got = np.concatenate([bb.cpu().numpy(), o.cpu().numpy()], 1)
    for u in range(U):
        if u == 1:
            continue  # zero f_TM: only the src0 half contributes
        assert normwise(got[u], ref[u]) <= TOL, u
    assert normwise(got[1], ref[1]) <= TOL


@pytest.mark.parametrize("Hin,Win", [(64, 64), (33, 47), (7, 5), (40, 70)])
def test_upsample2x_tiled_and_projection_order(Hin, Win):
    """tmr_upsample2x (LDS-tiled, 32x128 output tiles) bit-exact against the C
    restatement at tile-edge and W % 4 != 0 sizes; the engine's projection
    (input_proj at the features' size, then up2x) within the fp32 contract of
    ATen's conv2d(interpolate(f)) (matching_net.py:50-51,56)."""
    from tmr_amd._lib import call, ptr, stream
    torch.manual_seed(Hin * 100 + Win)
    C = 24
    f = torch.randn(2, C, Hin, Win)
    fd = cuda(f)
    out = torch.empty((2, C, 2 * Hin, 2 * Win), device=DEV)
    call("tmr_upsample2x", ptr(fd), 2 * C, Hin, Win, ptr(out), stream())
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), np.stack([oracle.upsample2x(x) for x in f.numpy()]))
    P = synth.reference_state_dict(3, cin=C, emb=40)
    ref = torch.nn.functional.conv2d(
        torch.nn.functional.interpolate(f, scale_factor=2, mode="bilinear", align_corners=False),
        P["input_proj.0.weight"], P["input_proj.0.bias"])
    eng = tmr_amd.TMREngine({k: cuda(v) for k, v in P.items()}, tmr_amd.PathConfig(emb_dim=40))
    fp, _ = eng.project(fd)
    assert normwise(fp.cpu().numpy(), ref.numpy()) <= TOL


def _xrecords_ref(x, ks, prec, xmax):
    """tmr_split_xpack's record layout restated in torch: [s][chunk][half]
    [piece q][Hp][Wp][8 x 16-bit], hi = fl16(x s), lo = fl16(x s - hi) (F16X3),
    s = 2^(14 - e) with max|x| < 2^e (conv_split.hip split_scale), zero ring."""
    S, C, H, W = x.shape
    NCc, pad = (C + 31) // 32, ks // 2
    Hp, Wp = -(-H // 16) * 16 + ks - 1, -(-W // 32) * 32 + ks - 1
    xs = torch.zeros(S, NCc * 32, Hp, Wp, dtype=torch.float32, device=x.device)
    sc = 1.0
    if prec != "bf16":  # one source, one per sample [S] or one per pixel [S,H,W]
        m = np.asarray(xmax, np.float32)
        e = np.frexp(m)[1]
        sc = np.where(m > 0, np.exp2(np.clip(14 - e, -63, 63)), 1.0).astype(np.float32)
        sc = torch.from_numpy(sc.reshape((S, 1, H, W) if m.ndim == 3 else (-1, 1, 1, 1) if m.ndim else ()))
        sc = sc.to(x.device)
    xs[:, :C, pad:pad + H, pad:pad + W] = x * sc
    dt = torch.bfloat16 if prec == "bf16" else torch.float16
    hi = xs.to(dt)
    halves = [hi]
    if prec == "fp32":
        halves.append((xs - hi.float()).to(dt))
    # [S][NCc][32][Hp][Wp] -> [S][NCc][P=4][Hp][Wp][8]
    recs = [h.view(S, NCc, 4, 8, Hp, Wp).permute(0, 1, 2, 4, 5, 3) for h in halves]
    return torch.stack(recs, 2).contiguous().view(torch.int16).flatten()


@pytest.mark.parametrize("S,C,H,W,ks", [(2, 40, 19, 36, 3), (1, 64, 128, 128, 3), (3, 33, 8, 12, 1),
                                        (2, 32, 9, 20, 5), (2, 40, 19, 37, 3), (1, 8, 16, 32, 1)])
def test_xpack_records_bitexact(S, C, H, W, ks):
    """Activation records (the 4-pixel kernel for W % 4 == 0, the one-pixel
    kernel otherwise) bit-exact against the torch restatement of the layout,
    padding ring included (the buffer is pre-filled with garbage)."""
    from tmr_amd._lib import PREC_CODES, call, ptr, size, stream
    from tmr_amd.engine import absmax, absmax_rows, pixel_absmax
    torch.manual_seed(11)
    # samples 2^20 apart and a quiet pixel block: the per-sample and per-pixel
    # scale modes (xmax_per_sample 1 / 2) are exercised with real spread
    x = (torch.randn(S, C, H, W) * 3 * torch.tensor([2.0 ** (-20 * s) for s in range(S)])[:, None, None, None])
    x[0, :, : H // 2, : W // 3] *= 1e-6
    x = x.cuda()
    for mode, xmax in ((0, absmax(x)), (1, absmax_rows(x)), (2, pixel_absmax(x))):
        for prec in ("fp32", "bf16", "f16"):
            n = size("xpack", S, C, H, W, ks, PREC_CODES[prec])
            out = torch.full((n,), 0x5A, device="cuda", dtype=torch.uint8)
            call("tmr_split_xpack", ptr(x), S, C, H, W, 0, ks, PREC_CODES[prec], ptr(xmax), mode, ptr(out),
                 stream())
            ref = _xrecords_ref(x, ks, prec, xmax.cpu().numpy() if mode else float(xmax.item()))
            got = out.view(torch.int16)
            assert got.numel() == ref.numel(), prec
            bad = int((got != ref).sum())
            assert bad == 0, f"{prec}: {bad} of {ref.numel()} 16-bit words differ"
            if prec == "bf16" and W % 8 == 0:
                # the bf16 input form (tmr_split_xpack16 of bf16(x), the bf16
                # f_TM plane of tmr_xcorr out_bf16): the same records bit for bit
                out16 = torch.full((n,), 0x5A, device="cuda", dtype=torch.uint8)
                xb = x.to(torch.bfloat16)
                call("tmr_split_xpack16", ptr(xb), S, C, H, W, ks, PREC_CODES[prec], ptr(out16), stream())
                assert torch.equal(out16, out), "xpack16"


def test_split_acc_slab_bf16():
    """The bf16 per-image fp-half slab of the bf16 contract (TMR_SPLIT_OUT_BF16
    on the store, TMR_SPLIT_INIT_BF16 on the heads launch): heads partials from
    a bf16 slab vs an fp32 slab of the same store (bf16 rounding of the
    initial values only), and vs the unsplit fp64 reference within the bf16
    contract; the flags are refused under the fp32 3-term split and without a
    tiled buffer."""
    from tmr_amd._lib import (PREC_CODES, SPLIT_INIT_BF16, SPLIT_OUT_BF16, SPLIT_TILED_INIT,
                              SPLIT_TILED_OUT, call, ptr, size, stream)
    from tmr_amd.engine import absmax, pack_split_w, pack_split_x
    torch.manual_seed(5)
    B, U, C0, C1, N, H, W = 2, 3, 40, 48, 136, 19, 37
    x0, x1 = torch.randn(B, C0, H, W), torch.randn(U, C1, H, W)
    ui = np.array([1, 0, 1], np.int32)
    w = torch.randn(N, C0 + C1, 3, 3) * 0.02
    bias = torch.randn(N) * 0.1
    hw = torch.zeros(((N + 127) // 128) * 128, 5)
    hw[:N] = torch.randn(N, 5)
    xcat = torch.cat([x0[torch.from_numpy(ui).long()], x1], 1)
    act = torch.nn.functional.leaky_relu(torch.nn.functional.conv2d(xcat.double(), w.double(),
                                                                    bias.double(), padding=1), 0.01)
    ref = torch.einsum("unhw,nj->ujhw", act, hw[:N].double()).numpy()
    d = {k: cuda(v) for k, v in dict(x0=x0, x1=x1, w0=w[:, :C0].contiguous(), w1=w[:, C0:].contiguous(),
                                     b=bias, hw=hw).items()}
    zero = torch.zeros(N, device=DEV)
    uid = cuda(torch.from_numpy(ui))
    pc = PREC_CODES["bf16"]
    wp0, wm0 = pack_split_w(d["w0"], C0, "bf16")
    wp1, wm1 = pack_split_w(d["w1"], 0, "bf16")
    xm0, xm1 = absmax(d["x0"]), absmax(d["x1"])
    xp0, xp1 = pack_split_x(d["x0"], 3, "bf16", xm0), pack_split_x(d["x1"], 3, "bf16", xm1)
    slabs = {}
    for tag, fl in (("fp32", 0), ("bf16", SPLIT_OUT_BF16)):
        slabs[tag] = torch.empty(size("acc", B, N, H, W), device=DEV)
        call("tmr_split_conv", ptr(xp0), C0, None, None, 0, B, H, W, 3, pc, ptr(wp0), ptr(wm0),
             ptr(xm0), ptr(zero), N, 0, None, None, ptr(slabs[tag]), SPLIT_TILED_OUT | fl, stream())
    got = {}
    for tag, fl in (("fp32", 0), ("bf16", SPLIT_INIT_BF16)):
        part = torch.empty(size("heads_partials", N, U, H, W), device=DEV)
        call("tmr_split_conv", None, 0, ptr(uid), ptr(xp1), C1, U, H, W, 3, pc, ptr(wp1), ptr(wm1),
             ptr(xm1), ptr(d["b"]), N, 1, ptr(d["hw"]), ptr(slabs[tag]), ptr(part), SPLIT_TILED_INIT | fl,
             stream())
        o, bb = torch.empty((U, 1, H, W), device=DEV), torch.empty((U, 4, H, W), device=DEV)
        call("tmr_heads_reduce", ptr(part), N, 128, U, H, W, ptr(torch.zeros(5, device=DEV)), ptr(o), ptr(bb),
             stream())
        torch.cuda.synchronize()
        got[tag] = np.concatenate([bb.cpu().numpy(), o.cpu().numpy()], 1)
    e_slab = normwise(got["bf16"], got["fp32"])
    e_ref = max(normwise(got["bf16"][u], ref[u]) for u in range(U))
    print(f"bf16 slab vs fp32 slab {e_slab:.2e}, vs fp64 reference {e_ref:.2e}")
    assert 0.0 < e_slab <= 1e-2 and e_ref <= SPLIT_TOL["bf16"]
    out = torch.empty(size("acc", B, N, H, W), device=DEV)
    wpf, wmf = pack_split_w(d["w0"], C0, "fp32")
    with pytest.raises(tmr_amd.TMRError):  # bf16 slabs are a one-term-precision layout
        call("tmr_split_conv", ptr(pack_split_x(d["x0"], 3, "fp32", xm0)), C0, None, None, 0, B, H, W, 3,
             PREC_CODES["fp32"], ptr(wpf), ptr(wmf), ptr(xm0), ptr(zero), N, 0, None, None, ptr(out),
             SPLIT_TILED_OUT | SPLIT_OUT_BF16, stream())
    with pytest.raises(tmr_amd.TMRError):  # OUT_BF16 needs the tiled output
        call("tmr_split_conv", ptr(xp0), C0, None, None, 0, B, H, W, 3, pc, ptr(wp0), ptr(wm0), ptr(xm0),
             ptr(zero), N, 0, None, None, ptr(out), SPLIT_OUT_BF16, stream())


def test_shared_and_unshared_fp_half_agree():
    """The decoder's fp half computed once per image (acc0 shared by the
    image's exemplars) and per unit in the same launch give the same maps
    within the fp32 contract, folded and unfolded projection both, and
    both match the oracle forward."""
    B, E = 2, 2
    P = synth.reference_state_dict(4, cin=64, emb=96, obj_bias=-0.3)
    feats_h = synth.sam_features(18, B, 64, 20, 23)
    feats = cuda(feats_h)
    ex, _ = synth.exemplar_set(19, B, E, 40, 46, 3, 9)
    ui = np.repeat(np.arange(B), E)
    res = {}
    for fold in (True, False):
        for share in (True, False):
            eng = tmr_amd.TMREngine({k: cuda(v) for k, v in P.items()}, tmr_amd.PathConfig(emb_dim=96))
            eng.fold_proj, eng.share_fp_half = fold, share
            r = eng.forward_units(feats, ui, ex.reshape(-1, 4))
            assert eng.last_decoder_algo == "split"
            assert (eng.last_shared_flops > 0) == share
            res[(fold, share)] = (r["o"].cpu().numpy(), r["b"].cpu().numpy())
    for u in range(B * E):
        ro, rb, _, _ = oracle.forward_torch(torch.from_numpy(feats_h[ui[u]:ui[u] + 1]),
                                            [torch.from_numpy(ex.reshape(-1, 4)[u:u + 1])], P)
        for k, (o, b) in res.items():
            assert normwise(o[u], ro[0][0].numpy()) <= TOL, (k, u)
            assert normwise(b[u], rb[0][0].numpy()) <= TOL, (k, u)


def test_heads_vs_torch():
    torch.manual_seed(1)
    x = torch.randn(3, 96, 20, 28)
    for cls in (tmr_amd.ObjectnessHead, tmr_amd.BboxesHead):
        h = cls(96)
        with torch.no_grad():
            h.head[0].bias.normal_()
        ref = h.head[0](x).detach().numpy()
        got = h.to(DEV)(x.to(DEV)).cpu().numpy()
        assert normwise(got, ref) <= TOL


# ----------------------------------------------------------------- forward
class _Passthrough(torch.nn.Module):
    def __init__(self, c):
        super().__init__()
        self.num_channels = c

    def forward(self, x):
        return x


@pytest.mark.parametrize("name", ["default", "squeeze", "prototype", "nofusion", "noboxreg",
                                  "twolayer_k5", "noupsample", "nomatcher"])
def test_matching_net_forward_golden(golden, name):
    from types import SimpleNamespace
    g = golden(f"forward_{name}")
    args = SimpleNamespace(**json.loads(str(g["args"])))
    model = tmr_amd.matching_net(_Passthrough(g["feats"].shape[1]), args)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    model.load_state_dict(sd, strict=True)
    model = model.to(DEV).eval()
    ex = [cuda(e) for e in g["exemplars"]]
    os_, bs_, ftm, f0 = model(cuda(g["feats"]), ex)
    assert normwise(os_[0].cpu().numpy(), g["o"]) <= TOL
    if "b" in g:
        assert normwise(bs_[0].cpu().numpy(), g["b"]) <= TOL
    else:
        assert bs_[0] is None
    assert normwise(ftm[0].cpu().numpy(), g["f_tm"]) <= TOL
    f0n = f0.cpu().numpy()
    assert normwise(f0n, g["f0"]) <= 1e-6
    if args.feature_upsample:  # the fma form is bit-exact with the C restatement
        assert bits_equal(f0n, np.stack([oracle.upsample2x(x) for x in g["feats"]]))


# ----------------------------------------------------------------- peaks
def _split(g, key):
    counts = g[key + "_counts"]
    out, o = [], 0
    for c in counts:
        out.append(g[key][o:o + c]); o += c
    return out


KERNELS = [[[1, 1, 1], [1, 1, 1], [1, 1, 1]], [[0, 0, 0], [0, 1, 0], [0, 0, 0]],
           [[0, 1, 0], [0, 1, 0], [0, 1, 0]], [[0, 0, 0], [1, 1, 1], [0, 0, 0]],
           [[0, 1, 0], [1, 1, 1], [0, 1, 0]], [[1, 0, 0], [0, 0, 0], [0, 0, 1]]]


def _maxpool_reference(x, kernel):
    """TM_utils.py:337-361 as written (F.unfold + mask + max), torch CPU."""
    import torch.nn.functional as F
    flat = torch.tensor(kernel, dtype=torch.bool).flatten()
    N, C, H, W = x.shape
    patches = F.unfold(x, kernel_size=3, padding=1).view(N, -1, 9, H, W)
    return patches[:, :, flat, :, :].max(dim=2)[0]


@pytest.mark.parametrize("shape", [(2, 3, 7, 9), (1, 1, 1, 1), (1, 2, 128, 128), (3, 1, 2, 5)])
def test_custom_shape_maxpool_vs_reference(shape):
    """Bit-exact against the reference formulation for every adaptive
    kernel shape (plus an off-centre one): negatives (the zero padding
    wins at the border), exact ties, +-0 and a NaN."""
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.round(torch.randn(shape, generator=g) * 4) / 4  # many exact ties
    x.view(-1)[::7] = -x.view(-1)[::7].abs() - 1
    if x.numel() > 20:
        x.view(-1)[5] = -0.0
        x.view(-1)[11] = float("nan")
    for k in KERNELS:
        ref = _maxpool_reference(x, k)
        got = tmr_amd.custom_shape_3x3_maxpool2d(x.to(DEV), k).cpu()
        assert got.shape == ref.shape
        assert torch.equal(torch.isnan(got), torch.isnan(ref)), k
        m = ~torch.isnan(ref)
        assert torch.equal(got[m], ref[m]), k
    with pytest.raises(tmr_amd.TMRError):
        tmr_amd.custom_shape_3x3_maxpool2d(x.to(DEV), [[0] * 3] * 3)


@pytest.mark.parametrize("name", ["pred_boxes", "pred_boxes_nonfinite"])
def test_get_pred_boxes_golden(golden, name):
    """Bit-exact given identical score maps: feed the reference's own
    sigmoid output (input_is_prob) and compare every candidate.  The
    _nonfinite fixture holds NaN at the first / last masked tap of would-be
    peaks, NaN centres, NaN beside plateaus, +-inf logits, a NaN regression
    value and an all-NaN map: the reference's torch.max propagates NaN
    (TM_utils.py:253,359), so no pixel with a NaN in its window is a peak."""
    g = golden(name)
    for i in range(int(g["n"])):
        meta = json.loads(str(g[f"c{i}_meta"]))
        prob, reg, ex = g[f"c{i}_prob"], g[f"c{i}_reg"], g[f"c{i}_ex"]
        batch = {"regression_ablation_b": meta["ab_b"], "regression_ablation_c": meta["ab_c"]}
        exl = [cuda(e[None]) for e in ex]
        regs = [cuda(reg)] if meta["box_reg"] else [None]
        L, Bx, R = tmr_amd.Get_pred_boxes([cuda(prob[:, None])], regs, exl, batch, meta["thr"],
                                          meta["box_reg"], input_is_prob=True)
        gL, gB, gR = _split(g, f"c{i}_logits"), _split(g, f"c{i}_boxes"), _split(g, f"c{i}_refs")
        oL, oB, oR = oracle.get_pred_boxes_prob(list(prob), list(reg) if meta["box_reg"] else None,
                                                [e[None] for e in ex], meta["thr"], meta["box_reg"],
                                                meta["ab_b"], meta["ab_c"])
        for b in range(len(gL)):
            l, bx, r = L[b].cpu().numpy(), Bx[b].cpu().numpy(), R[b].cpu().numpy()
            assert bits_equal(l, gL[b]), (i, b, meta)
            assert bits_equal(r, gR[b]), (i, b)
            assert bits_equal_nan(bx, gB[b]), (i, b)  # the reference's own decode, bit for bit
            assert bits_equal_nan(bx, oB[b]), (i, b)
        if name == "pred_boxes_nonfinite":
            # from the logits, the probability map discarded (the kernel's scratch
            # mode, detect's and Get_pred_boxes' default): the same candidates as the
            # oracle on the path's sigmoid of those logits
            o = g[f"c{i}_o"]
            L2, B2, R2 = tmr_amd.Get_pred_boxes([cuda(o)], regs, exl, batch, meta["thr"], meta["box_reg"])
            pl = oracle.sigmoid_cr(o[:, 0])
            qL, qB, qR = oracle.get_pred_boxes_prob(list(pl), list(reg) if meta["box_reg"] else None,
                                                    [e[None] for e in ex], meta["thr"], meta["box_reg"],
                                                    meta["ab_b"], meta["ab_c"])
            for b in range(len(qL)):
                assert bits_equal(L2[b].cpu().numpy(), qL[b]), (i, b, meta)
                assert bits_equal_nan(B2[b].cpu().numpy(), qB[b]), (i, b)
                assert bits_equal(R2[b].cpu().numpy(), qR[b]), (i, b)


def test_get_pred_boxes_empty_units_dummy_row():
    """A unit with no peak returns the reference's dummy row (TM_utils.py:
    288-291), which tmr_peaks_decode writes at the unit's row 0: values and
    shapes equal the oracle's, next to non-empty units, twice in a row (the
    row of a unit that had peaks the call before is rewritten)."""
    H = W = 32
    prob = np.full((3, H, W), 0.05, np.float32)
    prob[1, 10, 12] = 0.9  # unit 1 has one peak, units 0 and 2 none
    reg = synth.normal(91, (3, 4, H, W)) * 0.5
    ex = np.array([[0.1, 0.1, 0.3, 0.3], [0.2, 0.2, 0.5, 0.6], [0.4, 0.1, 0.6, 0.2]], np.float32)
    batch = {"regression_ablation_b": False, "regression_ablation_c": False}
    for order in ((0, 1, 2), (1, 0, 2)):
        p_, r_, e_ = prob[list(order)], reg[list(order)], ex[list(order)]
        L, Bx, R = tmr_amd.Get_pred_boxes([cuda(p_[:, None])], [cuda(r_)], [cuda(e[None]) for e in e_], batch,
                                          0.5, True, input_is_prob=True)
        oL, oB, oR = oracle.get_pred_boxes_prob(list(p_), list(r_), [e[None] for e in e_], 0.5, True, False, False)
        for b in range(3):
            assert L[b].dtype == torch.float32 and tuple(L[b].shape) == np.asarray(oL[b]).shape
            assert bits_equal(L[b].cpu().numpy(), oL[b]) and bits_equal(Bx[b].cpu().numpy(), oB[b])
            assert bits_equal(R[b].cpu().numpy(), oR[b])
        empty = [b for b in range(3) if order[b] != 1]
        for b in empty:
            assert np.array_equal(Bx[b].cpu().numpy(), np.array([[0, 0, 1e-14, 1e-14]], np.float32))


def _peaks_sweep_case(r):
    """One random Get_pred_boxes call: map shape (small, medium, one-row-wide
    up to 8192 columns, tall and narrow, several LDS chunks), unit count,
    logit law (near-ties around 0, plateaus, saturated, +-inf / NaN pixels),
    exemplar boxes from sub-pixel to most of the map (every adaptive kernel
    shape), threshold, box regression and the ablation flags."""
    law = r.integers(0, 4)
    if law == 0:
        H, W = int(r.integers(1, 41)), int(r.integers(1, 41))
    elif law == 1:
        H, W = int(r.integers(41, 301)), int(r.integers(41, 301))
    elif law == 2:
        H, W = int(r.integers(1, 5)), int(r.integers(300, 8193))
    else:
        H, W = int(r.integers(300, 2001)), int(r.integers(1, 5))
    U = int(r.integers(1, 7))
    sig = float(r.choice([0.05, 1.0, 3.0, 10.0]))
    o = (r.standard_normal((U, 1, H, W)) * sig).astype(np.float32)
    if r.random() < 0.5:  # plateaus: exact ties between neighbours
        q = float(r.choice([0.25, 1.0]))
        o = (np.round(o / q) * q).astype(np.float32)
    flat = o.reshape(-1)
    k = max(1, flat.size // 500)
    if r.random() < 0.3:
        flat[r.integers(0, flat.size, k)] = 30.0
    if r.random() < 0.3:
        flat[r.integers(0, flat.size, k)] = np.float32(r.choice([np.inf, -np.inf, np.nan]))
    reg = (r.standard_normal((U, 4, H, W)) * 0.5).astype(np.float32)
    x1, y1 = r.uniform(-0.1, 0.9, U), r.uniform(-0.1, 0.9, U)
    bw = 10.0 ** r.uniform(np.log10(0.25 / max(W, 1)), np.log10(0.8), U)
    bh = 10.0 ** r.uniform(np.log10(0.25 / max(H, 1)), np.log10(0.8), U)
    boxes = np.stack([x1, y1, x1 + bw, y1 + bh], 1).astype(np.float32)
    thr = float(r.uniform(0.01, 0.99))
    box_reg = bool(r.random() < 0.8)
    if r.random() < 0.1:  # thresholds near 1: logits across the band that rounds to thr
        thr = float(np.float32(1.0 - 10.0 ** -r.uniform(3.0, 7.2)))
        lg = np.log(thr / (1.0 - thr))
        sel = r.random(flat.size) < 0.3
        flat[sel] = (lg + r.uniform(-1.0, 1.0, int(sel.sum()))).astype(np.float32)
    ab = int(r.integers(0, 4))  # 0, 1: none; 2: ablation_b; 3: ablation_c
    return o, reg, boxes, thr, box_reg, ab == 2, ab == 3


def test_peaks_random_sweep_vs_oracle():
    """Seeded random Get_pred_boxes calls (TMR_PEAKS_SWEEP, default 60): every
    unit's candidate logits, boxes and reference points bit-exact vs the
    oracle on the correctly rounded sigmoid of the same logits (the call
    discards the probability map, so the kernel runs in its scratch mode)."""
    import os
    n = int(os.environ.get("TMR_PEAKS_SWEEP", "60"))
    r = np.random.default_rng(5151)
    npx = ncand = 0
    for i in range(n):
        o, reg, boxes, thr, box_reg, ab_b, ab_c = _peaks_sweep_case(r)
        batch = {"regression_ablation_b": ab_b, "regression_ablation_c": ab_c}
        L, Bx, R = tmr_amd.Get_pred_boxes([cuda(o)], [cuda(reg)] if box_reg else None,
                                          [cuda(b[None]) for b in boxes], batch, thr, box_reg)
        prob = oracle.sigmoid_cr(o)
        oL, oB, oR = oracle.get_pred_boxes_prob(list(prob[:, 0]), list(reg) if box_reg else None,
                                                [b[None] for b in boxes], thr, box_reg, ab_b, ab_c)
        for b in range(len(boxes)):
            meta = (i, b, o.shape, thr, box_reg, ab_b, ab_c)
            assert bits_equal(L[b].cpu().numpy(), oL[b]), meta
            assert bits_equal(Bx[b].cpu().numpy(), oB[b]), meta
            assert bits_equal(R[b].cpu().numpy(), oR[b]), meta
            ncand += len(oL[b])
        npx += o.size
    print(f"peaks sweep: {n} calls, {npx} pixels, {ncand} candidates")


def test_peaks_large_random_vs_oracle():
    """128x128 maps with plateaus, saturation, every kernel shape; bit-exact."""
    H = W = 128
    o = synth.normal(77, (6, 1, H, W)) * 3.0
    o[0, 0, 10:20, 10:20] = 2.0
    o[1, 0, 50:52, :] = 30.0
    reg = synth.normal(78, (6, 4, H, W)) * 0.5
    boxes = np.array([[0.1, 0.1, 0.3, 0.3], [0.1, 0.1, 0.1 + 1 / 256, 0.1 + 1 / 256],
                      [0.1, 0.1, 0.2, 0.1 + 1 / 256], [0.1, 0.1, 0.1 + 1 / 256, 0.2],
                      [0.1, 0.1, 0.1 + 2.5 / 128, 0.1 + 2.5 / 128], [-0.1, 0.4, 0.2, 1.2]], np.float32)
    prob = oracle.sigmoid_cr(o)
    for thr in (0.1, 0.7):
        batch = {"regression_ablation_b": False, "regression_ablation_c": False}
        L, Bx, R = tmr_amd.Get_pred_boxes([cuda(o)], [cuda(reg)], [cuda(b[None]) for b in boxes],
                                          batch, thr, True)
        oL, oB, oR = oracle.get_pred_boxes_prob(list(prob[:, 0]), list(reg), [b[None] for b in boxes],
                                                thr)
        for b in range(6):
            assert bits_equal(L[b].cpu().numpy(), oL[b]), (thr, b)
            assert bits_equal(Bx[b].cpu().numpy(), oB[b]), (thr, b)
            assert bits_equal(R[b].cpu().numpy(), oR[b]), (thr, b)


# ----------------------------------------------------------------- nms
@pytest.mark.parametrize("name", ["nms", "nms_nonfinite"])
def test_nms_golden(golden, name):
    """Keep lists and kept rows vs the reference's NMS.  _nonfinite: NaN
    scores of either sign sort first (torch.sort descending, stable), +-inf
    scores, -0.0 == +0.0 ties, NaN / inf coordinates; 8-row sets (one
    workgroup) and 300 / 700-row sets (radix sort + binned pairs)."""
    g = golden(name)
    for i in range(int(g["n"])):
        bx, sc, thr = g[f"c{i}_boxes"], g[f"c{i}_scores"], float(g[f"c{i}_thr"])
        keep = tmr_amd.NMS_process(cuda(bx), cuda(np.stack([sc, np.zeros_like(sc)], 1)), thr)
        assert np.array_equal(keep.cpu().numpy(), g[f"c{i}_keep"]), i
        if bx.shape[0]:
            L, B, R = tmr_amd.NMS([cuda(np.stack([sc, np.zeros_like(sc)], 1))], [cuda(bx)],
                                  [cuda(bx[:, :2].copy())], thr)
            assert bits_equal(B[0].cpu().numpy(), g[f"c{i}_kept_boxes"]), i
            if f"c{i}_kept_logits" in g:
                assert bits_equal(L[0].cpu().numpy(), g[f"c{i}_kept_logits"]), i


@pytest.mark.parametrize("n,thr", [(1, 0.5), (63, 0.5), (64, 0.15), (65, 0.5), (700, 0.5),
                                   (3000, 0.5), (5000, 0.15)])
def test_nms_random_vs_oracle(n, thr):
    u = synth.uniform(n, 5 * n).reshape(n, 5).astype(np.float32)
    xy = u[:, :2] * 0.9
    bx = np.concatenate([xy, xy + 0.01 + u[:, 2:4] * 0.1], 1).astype(np.float32)
    sc = (np.round(u[:, 4] * 64) / 64).astype(np.float32)  # ties
    keep = tmr_amd.NMS_process(cuda(bx), cuda(np.stack([sc, np.zeros_like(sc)], 1)), thr)
    assert np.array_equal(keep.cpu().numpy(), oracle.nms(bx, sc, thr))


def _nms_case(seed, n):
    u = synth.uniform(seed, 5 * n).reshape(n, 5).astype(np.float32)
    xy = u[:, :2] * 0.5
    bx = np.concatenate([xy, xy + 0.01 + u[:, 2:4] * 0.3], 1).astype(np.float32)
    sc = (np.round(u[:, 4] * 16) / 16).astype(np.float32)  # many ties
    return bx, sc


def test_nms_small_images_one_workgroup_path():
    """Calls whose images all hold <= 256 candidates run the one-workgroup
    kernel; a call with a larger image runs gather + radix sort + strips for
    every image.  The same image gives the same kept rows and order either
    way -- ties, duplicate boxes, zero-area boxes, -0.0 / +0.0 and NaN
    scores included -- and equals the oracle (NaN scores sort first)."""
    big_bx, big_sc = _nms_case(501, 900)
    for seed, n in ((502, 1), (503, 17), (504, 64), (505, 65), (506, 200), (507, 256)):
        bx, sc = _nms_case(seed, n)
        if n >= 17:
            bx[3] = bx[5]; sc[3] = sc[5]  # duplicate row
            bx[7, 2:] = bx[7, :2]  # zero area
            sc[8], sc[9] = -0.0, 0.0
        for with_nan in (False, True):
            s2 = sc.copy()
            if with_nan and n >= 17:
                s2[11] = np.nan
            lg = np.stack([s2, np.zeros_like(s2)], 1)
            lgb = np.stack([big_sc, np.zeros_like(big_sc)], 1)
            for thr in (0.15, 0.5):
                L1, B1, R1 = tmr_amd.NMS([cuda(lg)], [cuda(bx)], [cuda(bx[:, :2].copy())], thr)
                L2, B2, R2 = tmr_amd.NMS([cuda(lg), cuda(lgb)], [cuda(bx), cuda(big_bx)],
                                         [cuda(bx[:, :2].copy()), cuda(big_bx[:, :2].copy())], thr)
                assert bits_equal(L1[0].cpu().numpy(), L2[0].cpu().numpy()), (n, with_nan, thr)
                assert bits_equal(B1[0].cpu().numpy(), B2[0].cpu().numpy()), (n, with_nan, thr)
                assert bits_equal(R1[0].cpu().numpy(), R2[0].cpu().numpy()), (n, with_nan, thr)
                keep = oracle.nms(bx, s2, thr)  # NaN scores first, as torch.sort(descending)
                assert bits_equal(B1[0].cpu().numpy(), bx[keep]), (n, with_nan, thr)


def _nms_binned_cases():
    """Images that stress the spatially binned NMS (csrc/nms.hip): a uniform
    spray of small boxes, a cluster of identical boxes (every row suppresses
    the rest: the lists overflow CAP and kept rows rescan their window),
    tiny and huge boxes mixed, boxes touching exactly edge to edge, inverted
    and zero-area boxes, far-from-origin coordinates, score ties."""
    r = np.random.default_rng(77)
    cases = []
    n = 1500
    xy = r.random((n, 2), np.float32) * 0.95
    wh = (0.005 + r.random((n, 2)) * 0.04).astype(np.float32)
    cases.append(np.concatenate([xy, xy + wh], 1))
    base = np.array([0.4, 0.4, 0.45, 0.47], np.float32)
    cl = np.repeat(base[None], 400, 0)
    cl[200:] += (r.random((200, 1)) * 0.01).astype(np.float32)
    cases.append(cl)
    xy = r.random((n, 2), np.float32)
    wh = np.where(r.random((n, 1)) < 0.05, 0.3 + r.random((n, 2)) * 0.6, 0.002 + r.random((n, 2)) * 0.01)
    cases.append(np.concatenate([xy, xy + wh.astype(np.float32)], 1).astype(np.float32))
    g = np.arange(30, dtype=np.float32) / 32.0  # a grid of unit cells touching exactly
    gx, gy = np.meshgrid(g, g)
    t = np.stack([gx.ravel(), gy.ravel(), gx.ravel() + 1.0 / 32.0, gy.ravel() + 1.0 / 32.0], 1)
    t = np.concatenate([t, t[::3] + np.float32(1.0 / 64.0)])
    cases.append(t.astype(np.float32))
    xy = r.random((800, 2), np.float32) * 0.9
    bx = np.concatenate([xy, xy + 0.03], 1).astype(np.float32)
    bx[::7, 2] = bx[::7, 0] - 0.01   # inverted
    bx[1::11, 2:] = bx[1::11, :2]    # zero area
    cases.append(bx)
    xy = 1000.0 + r.random((700, 2), np.float32) * 3.0
    cases.append(np.concatenate([xy, xy + 0.05 + r.random((700, 2), np.float32) * 0.2], 1).astype(np.float32))
    out = []
    for k, bx in enumerate(cases):
        sc = (np.round(r.random(len(bx)) * 32) / 32).astype(np.float32)  # ties
        out.append((bx.astype(np.float32), sc))
    return out


@pytest.mark.parametrize("thr", [0.0, 0.15, 0.5, 0.9, -0.1])
def test_nms_binned_edge_cases_vs_oracle(thr):
    """The binned NMS (images above TMR_NMS_SMALL candidates) keeps exactly
    the oracle's sequential torchvision list on every case, all images of
    the call binned together (a negative threshold: one cell per image,
    every pair evaluated)."""
    cases = _nms_binned_cases()
    L, Bx, R = tmr_amd.NMS([cuda(np.stack([sc, np.zeros_like(sc)], 1)) for bx, sc in cases],
                           [cuda(bx) for bx, sc in cases], [cuda(bx[:, :2].copy()) for bx, sc in cases], thr)
    for k, (bx, sc) in enumerate(cases):
        keep = oracle.nms(bx, sc, thr)
        assert bits_equal(Bx[k].cpu().numpy(), bx[keep]), (thr, k, len(keep), Bx[k].shape[0])
        assert bits_equal(L[k].cpu().numpy()[:, 0], sc[keep]), (thr, k)


def _nms_threshold_cases():
    """Images for the threshold-narrowed windows (nms.hip window(): IoU > t
    bounds the corner offset by (1 - t) max(w_i, w_j) and w_j by w_i / t):
    box pairs shifted to IoU = t within a few ulps either side, nested
    boxes at area ratio ~ t, sizes spread over 1000x in one image, identical
    and near-identical boxes, very small and very large boxes."""
    r = np.random.default_rng(91)
    cases = []
    for t in (0.3, 0.5, 0.7, 0.99):
        n = 300
        xy = (r.random((n, 2)) * 0.8).astype(np.float32)
        sd = (0.01 + r.random((n, 1)) * 0.1).astype(np.float32)
        a = np.concatenate([xy, xy + sd], 1).astype(np.float32)
        d = sd[:, 0] * np.float32((1 - t) / (1 + t))  # IoU((s - d) / (s + d)) = t
        d = np.nextafter(d, np.where(r.random(n) < 0.5, 0, 1).astype(np.float32))
        bsh = a.copy()
        bsh[:, 0] += d
        bsh[:, 2] += d
        k = r.integers(0, 2, n)  # or shifted left / up
        bsh[k == 1] = a[k == 1] - np.stack([d * 0, d, d * 0, d], 1)[k == 1]
        cases.append(np.concatenate([a, bsh]).astype(np.float32))
    xy = r.random((900, 2), np.float32) * 0.7
    side = (10.0 ** r.uniform(-3.5, -0.5, (900, 1))).astype(np.float32)
    nest = np.concatenate([xy, xy + side], 1).astype(np.float32)
    inner = nest[::2].copy()
    f = np.sqrt(r.uniform(0.2, 0.9, (inner.shape[0], 1))).astype(np.float32)
    inner[:, 2:] = inner[:, :2] + (inner[:, 2:] - inner[:, :2]) * f
    cases.append(np.concatenate([nest, inner, nest[:50]]).astype(np.float32))  # + exact duplicates
    xy = r.random((600, 2), np.float32) * 1e-15
    cases.append(np.concatenate([xy, xy + 1e-17 + r.random((600, 2), np.float32) * 3e-16], 1).astype(np.float32))
    xy = r.random((600, 2), np.float32) * 1e20
    cases.append(np.concatenate([xy, xy + 1e18 + r.random((600, 2), np.float32) * 3e19], 1).astype(np.float32))
    out = []
    for bx in cases:
        sc = (np.round(r.random(len(bx)) * 64) / 64).astype(np.float32)
        out.append((bx, sc))
    return out


@pytest.mark.parametrize("thr", [1e-4, 3e-4, 0.3, 0.5, 0.7, 0.99, 1.0, 1.5])
def test_nms_threshold_windows_vs_oracle(thr):
    """The windows narrowed by the threshold miss no suppressing pair: keep
    lists bit-exact vs the oracle on boundary pairs (IoU = t +- ulps), nested
    boxes, 1000x size spreads, duplicates, tiny and huge boxes, thresholds
    below the narrowing cut-off (2^-12) and at / above 1."""
    cases = _nms_threshold_cases()
    L, Bx, R = tmr_amd.NMS([cuda(np.stack([sc, np.zeros_like(sc)], 1)) for bx, sc in cases],
                           [cuda(bx) for bx, sc in cases], [cuda(bx[:, :2].copy()) for bx, sc in cases], thr)
    for k, (bx, sc) in enumerate(cases):
        keep = oracle.nms(bx, sc, thr)
        assert bits_equal(Bx[k].cpu().numpy(), bx[keep]), (thr, k, len(keep), Bx[k].shape[0])
        assert bits_equal(L[k].cpu().numpy()[:, 0], sc[keep]), (thr, k)


def _nms_sweep_image(r):
    """One random image for the NMS sweep: a random count (small path and
    binned path), box-size law (narrow, spread over decades, thin in one
    axis, clustered near-duplicates), coordinate scale and offset, and score
    quantisation (ties)."""
    n = int(np.exp(r.uniform(np.log(2), np.log(20000))))
    law = r.integers(0, 4)
    xy = r.random((n, 2))
    if law == 0:
        wh = 0.003 + r.random((n, 2)) * 0.05
    elif law == 1:
        wh = 10.0 ** r.uniform(-3.5, -0.3, (n, 2))
    elif law == 2:  # thin boxes: one side up to 200x the other
        s = 10.0 ** r.uniform(-3, -1, (n, 1))
        a = 10.0 ** r.uniform(-2.3, 0, (n, 1))
        wh = np.where(r.random((n, 1)) < 0.5, np.concatenate([s, s * a], 1), np.concatenate([s * a, s], 1))
    else:  # clusters of near-duplicates around a few centres
        c = r.random((max(1, n // 50), 2))
        xy = c[r.integers(0, len(c), n)] + r.normal(0, 0.004, (n, 2))
        wh = 0.02 + r.random((n, 2)) * 0.01
    scale = 10.0 ** r.uniform(-4, 4)
    off = r.uniform(-1, 1) * scale * 10 ** r.integers(0, 3)
    bx = (np.concatenate([xy, xy + wh], 1) * scale + off).astype(np.float32)
    q = 2.0 ** r.integers(3, 24)
    sc = (np.round(r.random(n) * q) / q).astype(np.float32)
    return bx, sc


def test_nms_random_sweep_vs_oracle():
    """Seeded random calls (1-4 images each, TMR_NMS_SWEEP calls, default 60):
    every image's keep list bit-exact vs the oracle's sequential torchvision
    list, for a threshold drawn uniformly in (0, 1) per call (plus a few at
    the narrowing cut-off 2^-12 and at 0.999)."""
    import os
    ncalls = int(os.environ.get("TMR_NMS_SWEEP", "60"))
    r = np.random.default_rng(4242)
    worst = 0
    for call in range(ncalls):
        thr = float(r.choice([2.0 ** -12, 0.999])) if call % 10 == 9 else float(r.uniform(0.001, 0.999))
        imgs = [_nms_sweep_image(r) for _ in range(int(r.integers(1, 5)))]
        L, Bx, R = tmr_amd.NMS([cuda(np.stack([sc, np.zeros_like(sc)], 1)) for bx, sc in imgs],
                               [cuda(bx) for bx, sc in imgs], [cuda(bx[:, :2].copy()) for bx, sc in imgs], thr)
        for k, (bx, sc) in enumerate(imgs):
            keep = oracle.nms(bx, sc, thr)
            assert bits_equal(Bx[k].cpu().numpy(), bx[keep]), (call, thr, k, len(bx), len(keep), Bx[k].shape[0])
            assert bits_equal(L[k].cpu().numpy()[:, 0], sc[keep]), (call, thr, k)
            worst = max(worst, len(bx))
    print(f"nms sweep: {ncalls} calls, largest image {worst} candidates")


def test_nms_binned_nonfinite_boxes_match_dense():
    """Non-finite box coordinates put the image in one bin (every pair
    evaluated with the kernels' own fmaxf/fminf arithmetic): an image of
    <= 256 candidates gives the same kept rows through the one-workgroup
    path and through the binned path (called beside a large image)."""
    big_bx, big_sc = _nms_case(601, 900)
    for seed in (602, 603):
        bx, sc = _nms_case(seed, 200)
        bx[5, 0] = np.nan
        bx[9, 2] = np.inf
        bx[13, 1] = -np.inf
        lg = np.stack([sc, np.zeros_like(sc)], 1)
        lgb = np.stack([big_sc, np.zeros_like(big_sc)], 1)
        for thr in (0.15, 0.5):
            L1, B1, R1 = tmr_amd.NMS([cuda(lg)], [cuda(bx)], [cuda(bx[:, :2].copy())], thr)
            L2, B2, R2 = tmr_amd.NMS([cuda(lg), cuda(lgb)], [cuda(bx), cuda(big_bx)],
                                     [cuda(bx[:, :2].copy()), cuda(big_bx[:, :2].copy())], thr)
            assert bits_equal(L1[0].cpu().numpy(), L2[0].cpu().numpy()), (seed, thr)
            assert bits_equal(B1[0].cpu().numpy(), B2[0].cpu().numpy()), (seed, thr)


# ----------------------------------------------------------------- callers
def test_caller_sequence_golden(golden):
    """demo.Inference.infer / each_step_multi_exemplars through TMREngine.detect."""
    g = golden("caller")
    sd = {k[3:]: cuda(v) for k, v in g.items() if k.startswith("sd.")}
    eng = tmr_amd.TMREngine(sd, tmr_amd.PathConfig(emb_dim=16))
    for thr, iou in ((0.1, 0.5), (0.5, 0.15), (0.7, 0.5)):
        L, Bx, R = eng.detect(cuda(g["feats"]), g["exemplars"], thr, iou)
        tag = f"t{int(thr * 100)}_i{int(iou * 100)}"
        gl, gb = g[f"{tag}_logits"], g[f"{tag}_boxes"]
        assert L[0].shape == gl.shape, (tag, L[0].shape, gl.shape)
        assert np.allclose(L[0].cpu().numpy(), gl, rtol=0, atol=1e-6)
        assert np.allclose(Bx[0].cpu().numpy(), gb, rtol=1e-5, atol=1e-6)  # GPU maps (fp32 contract)
        assert bits_equal(R[0].cpu().numpy(), g[f"{tag}_refs"])


def test_shared_fp_half_matches_unshared():
    """conv(cat[fp,f_TM]) computed as conv_fp (once per image) + conv_tm (per
    unit) agrees with the single fused conv within the fp32 contract."""
    B, E = 2, 3
    P = synth.reference_state_dict(3, cin=64, emb=128, obj_bias=-0.5)
    feats = cuda(synth.sam_features(8, B, 64, 32, 32))
    ex, _ = synth.exemplar_set(9, B, E, 64, 64, 3, 11)
    eng = tmr_amd.TMREngine({k: cuda(v) for k, v in P.items()}, tmr_amd.PathConfig(emb_dim=128))
    ui = np.repeat(np.arange(B), E)
    r1 = eng.forward_units(feats, ui, ex.reshape(-1, 4))
    assert eng.last_shared_flops > 0
    eng.share_fp_half = False
    r0 = eng.forward_units(feats, ui, ex.reshape(-1, 4))
    assert eng.last_shared_flops == 0
    assert normwise(r1["o"].cpu().numpy(), r0["o"].cpu().numpy()) <= TOL
    assert normwise(r1["b"].cpu().numpy(), r0["b"].cpu().numpy()) <= TOL


@pytest.mark.parametrize("hf,E,kmin,kmax,thr,iou", [(64, 3, 3, 15, 0.1, 0.5),    # config B shape
                                                     (96, 3, 17, 31, 0.25, 0.5),  # config E shape (192^2)
                                                     (64, 1, 5, 9, 0.4, 0.5)])    # config D (RPINE, E=1)
def test_scripted_config_vs_oracle(hf, E, kmin, kmax, thr, iou):
    """Full scripted shapes (emb 512, SAM 256 x hf x hf -> 2hf x 2hf maps): fp32
    maps within 1e-5 of the torch-CPU oracle; then, given the GPU's own
    probability maps, peaks and NMS bit-exact against the C oracle."""
    B = 1
    Hm = 2 * hf
    P = oracle.reference_weights(0)
    P["objectness_head.head.0.bias"] = torch.tensor([-1.0])
    feats = synth.sam_features(5, B, 256, hf, hf)
    ex, ks = synth.exemplar_set(6 + hf, B, E, Hm, Hm, kmin, kmax)
    eng = tmr_amd.TMREngine({k: cuda(v) for k, v in P.items()}, tmr_amd.PathConfig())
    ui = np.repeat(np.arange(B), E)
    r = eng.forward_units(cuda(feats), ui, ex.reshape(-1, 4))
    o, b = r["o"].cpu().numpy(), r["b"].cpu().numpy()
    for u in range(B * E):
        exm = [torch.from_numpy(ex.reshape(-1, 4)[u:u + 1])]
        ro, rb, _, _ = oracle.forward_torch(torch.from_numpy(feats[ui[u]:ui[u] + 1]), exm, P)
        assert normwise(o[u], ro[0][0].numpy()) <= TOL
        assert normwise(b[u], rb[0][0].numpy()) <= TOL
    params = host.peak_params(ex.reshape(-1, 4), Hm, Hm, thr)
    logits, box, ref, counts, prob = tmr_amd.TMREngine.peaks(r["o"], r["b"], params)
    prob_h = prob.cpu().numpy()
    assert bits_equal(prob_h, oracle.sigmoid_cr(o[:, 0]))
    counts_h = counts.cpu().numpy()
    cands = []
    for u in range(B * E):
        _, lg, bx, rf = oracle.peaks_decode(prob_h[u], b[u], ex.reshape(-1, 4)[u], thr)
        assert counts_h[u] == lg.shape[0]
        s = u * Hm * Hm
        assert bits_equal(logits[s:s + counts_h[u]].cpu().numpy(), lg)
        assert bits_equal(box[s:s + counts_h[u]].cpu().numpy(), bx)
        cands.append((lg, bx, rf) if lg.shape[0] else (oracle.DUMMY_LOGITS, oracle.DUMMY_BOXES,
                                                        oracle.DUMMY_REFS))
    unit_off = torch.arange(B * E, device=DEV, dtype=torch.int64) * (Hm * Hm)
    L, Bx, R = tmr_amd.TMREngine.nms(logits, box, ref, counts, counts_h, unit_off,
                                      np.arange(0, B * E + 1, E), iou)
    ol, ob, orf = oracle.nms_lists([np.concatenate([c[0] for c in cands])],
                                   [np.concatenate([c[1] for c in cands])],
                                   [np.concatenate([c[2] for c in cands])], iou)
    assert bits_equal(L[0].cpu().numpy(), ol[0])
    assert bits_equal(Bx[0].cpu().numpy(), ob[0])
    assert bits_equal(R[0].cpu().numpy(), orf[0])


def test_detect_large_exemplar_count():
    """16 exemplars per image (config E fan-out) through TMREngine.detect:
    every image's union and keep list equal the oracle's NMS over the GPU's
    own candidates."""
    B, E, hf = 2, 16, 24
    P = synth.reference_state_dict(7, cin=32, emb=64, obj_bias=-0.2)
    feats = cuda(synth.sam_features(21, B, 32, hf, hf))
    ex, _ = synth.exemplar_set(22, B, E, 2 * hf, 2 * hf, 1, 31)
    eng = tmr_amd.TMREngine({k: cuda(v) for k, v in P.items()}, tmr_amd.PathConfig(emb_dim=64))
    L, Bx, R = eng.detect(feats, ex, 0.3, 0.5)
    r = eng.forward_units(feats, np.repeat(np.arange(B), E), ex.reshape(-1, 4))
    o, bb = r["o"].cpu().numpy(), r["b"].cpu().numpy()
    for img in range(B):
        ls, bs, rs = [], [], []
        for e in range(E):
            u = img * E + e
            prob = oracle.sigmoid_cr(o[u, 0])
            l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [bb[u]], [ex[img, e:e + 1]], 0.3)
            ls.append(l_[0]); bs.append(b_[0]); rs.append(r_[0])
        ol, ob, orf = oracle.nms_lists([np.concatenate(ls)], [np.concatenate(bs)],
                                       [np.concatenate(rs)], 0.5)
        assert bits_equal(L[img].cpu().numpy(), ol[0])
        assert bits_equal(Bx[img].cpu().numpy(), ob[0])


@pytest.mark.parametrize("prec", ["bf16", "f16"])
def test_reduced_precision_forward_vs_oracle(prec):
    """Config-C style reduced-precision decoders (one 16-bit MFMA term, fp32
    accumulation) at the scripted shape (emb 512, 128^2 maps, E=3), the
    correlation on the one-term MFMA kernel too: o and b within the stated
    normwise tolerance of the fp32 torch-CPU oracle."""
    B, E, hf = 1, 3, 64
    P = oracle.reference_weights(0)
    P["objectness_head.head.0.bias"] = torch.tensor([-1.0])
    feats = synth.sam_features(5, B, 256, hf, hf)
    ex, _ = synth.exemplar_set(70, B, E, 2 * hf, 2 * hf, 3, 15)
    eng = tmr_amd.TMREngine({k: cuda(v) for k, v in P.items()}, tmr_amd.PathConfig(precision=prec))
    eng.xcorr_algo = "mfma"
    ui = np.repeat(np.arange(B), E)
    r = eng.forward_units(cuda(feats), ui, ex.reshape(-1, 4))
    assert eng.last_decoder_algo == "split" and eng.last_xcorr_algo == "mfma"
    o, b = r["o"].cpu().numpy(), r["b"].cpu().numpy()
    for u in range(B * E):
        exm = [torch.from_numpy(ex.reshape(-1, 4)[u:u + 1])]
        ro, rb, _, _ = oracle.forward_torch(torch.from_numpy(feats[ui[u]:ui[u] + 1]), exm, P)
        eo, eb = normwise(o[u], ro[0][0].numpy()), normwise(b[u], rb[0][0].numpy())
        print(f"reduced precision {prec} unit {u}: normwise o {eo:.3e} b {eb:.3e}")
        assert eo <= SPLIT_TOL[prec] and eb <= SPLIT_TOL[prec]


# ----------------------------------------------------------------- xcorr (MFMA)
@pytest.mark.parametrize("H,W,C,kmax", [(128, 128, 16, 31), (70, 64, 24, 15), (70, 128, 8, 31),
                                        (192, 192, 8, 31), (33, 64, 8, 15), (128, 128, 8, 15),
                                        (100, 192, 8, 21), (77, 256, 8, 9), (40, 256, 8, 29)])
def test_xcorr_mfma_vs_oracle(H, W, C, kmax):
    """The row-Toeplitz MFMA correlation kernel (TMR_XCORR_MFMA, 3-term fp16
    split) against the C oracle at every odd template side 1..31, rectangular
    templates, several units per image, band edges (H % 32 / % 64 != 0), a
    learned scale, relu output, the fused max |f_TM| and the zero pad border.
    Both band heights run: 64-row bands where the band and halo fit the
    staging registers (W 64 / 128, W 192 with kmax <= 21, W 256 with kmax <=
    1), 32-row bands otherwise; every accumulator width (1-4 64-column
    groups)."""
    _xcorr_mfma_case(H, W, C, kmax, "fp32")


# bf16 MFMA path (BASELINE config C, north_star "within a stated bf16
# tolerance"): one bf16 term per product, fp32 accumulation -- SURVEY.md 8d's
# bf16 contract 1e-2 normwise (measured bf16 15x15 xcorr: 2.2e-3); one scaled
# fp16 term: 2e-3 (11-bit operands)
XCORR_ONE_TERM_TOL = {"bf16": 1e-2, "f16": 2e-3}


@pytest.mark.parametrize("prec", ["bf16", "f16"])
@pytest.mark.parametrize("H,W,C,kmax", [(128, 128, 16, 31), (70, 64, 24, 15), (128, 128, 8, 15),
                                        (100, 192, 8, 21)])
def test_xcorr_mfma_one_term_vs_oracle(H, W, C, kmax, prec):
    """tmr_xcorr with one bf16 / fp16 MFMA term: the same shapes, border,
    relu and fused-max contract as the 3-term kernel, at the one-term tolerance;
    the VALU kernel in the same call stays fp32 (1e-5)."""
    _xcorr_mfma_case(H, W, C, kmax, prec)


XCORR_SWEEP = int(os.environ.get("TMR_XCORR_SWEEP", "24"))


@pytest.mark.parametrize("seed", range(XCORR_SWEEP))
def test_xcorr_mfma_random_sweep_vs_oracle(seed):
    """Seeded random sweep of the 2-D window MFMA correlation (round 6) against
    the C oracle, away from the fixed shapes above: 1-3 images, 1-6 units with
    random image assignment (images without units included), every
    accumulator width (W 64 / 128 / 192 / 256), heights 1-160 (band edges at
    every residue), random odd rectangular templates up to the kernel's
    staging limit at random positions, feature scales 1e-6 ... 1e6, sparse and
    constant maps, a random learned scale; fp32 (3-term split, 1e-5 normwise)
    or one bf16 term (1e-2).  The fused per-unit max and relu output are
    checked bit for bit against the plane.  TMR_XCORR_SWEEP=N for more."""
    from tmr_amd._lib import PREC_CODES, XCORR_ALGOS, call, ptr, size, stream, xcorr
    from tmr_amd.engine import _h2d, _units_to_device
    r = np.random.default_rng(9000 + seed)
    B = int(r.integers(1, 4))
    W = int(r.choice([64, 128, 192, 256]))
    H = int(r.integers(1, 161))
    C = int(r.integers(1, 7))
    prec = "bf16" if r.random() < 0.2 else "fp32"
    kcap = 29 if W == 256 else 31  # (35 + 2 * (kmax // 2)) * W staged floats <= 16384
    f = synth.normal(7000 + seed, (B, C, H, W)) * np.float32(10.0 ** r.uniform(-6, 6))
    kind = r.integers(0, 4)
    if kind == 1:  # sparse
        f = f * (synth.uniform(7100 + seed, B * C * H * W).reshape(f.shape) < 0.05)
    elif kind == 2:  # constant planes
        f = np.broadcast_to(f[:, :, :1, :1], f.shape).copy()
    f = np.ascontiguousarray(f, np.float32)
    U = int(r.integers(1, 7))
    ui = sorted(int(x) for x in r.integers(0, B, U))
    boxes = []
    for u in range(U):
        kh = int(min(kcap, H // 2 * 2 - 1 if H % 2 == 0 else H, 2 * r.integers(0, 16) + 1))
        kw = int(min(kcap, 2 * r.integers(0, 16) + 1))
        boxes.append(synth.exemplar_box(kh, H, W, int(r.integers(0, H - kh + 1)), int(r.integers(0, W - kw + 1)), kw))
    boxes = np.stack(boxes)
    units, tfl, mh, mw = host.build_units(boxes, ui, H, W, C)
    fd = cuda(f)
    tm = tmr_amd.TemplateMatching("roi_align").to(DEV)
    tmpl = torch.cat([tm.extract_template(fd[ui[u]:ui[u] + 1], torch.from_numpy(boxes[u])).reshape(-1)
                      for u in range(U)])
    ud = _units_to_device(units, DEV)
    iu = _h2d(host.image_ranges(ui, B), DEV)
    sc = float(np.float32(r.uniform(0.2, 3.0)))
    scale = torch.tensor([sc], device=DEV)
    rows = host.tsplit_rows(units)
    tsplit = torch.empty(size("template_split", U, C, rows), device=DEV, dtype=torch.uint8)
    pc = PREC_CODES[prec]
    call("tmr_template_split", ptr(tmpl), ptr(ud), U, C, rows, pc, ptr(tsplit), stream())
    out = torch.empty((U, C, H, W), device=DEV)
    relu = torch.empty_like(out)
    amax = torch.zeros(U, device=DEV)
    xcorr(f=ptr(fd), templates=ptr(tmpl), units=ptr(ud), img_units=ptr(iu), scale=ptr(scale), out=ptr(out),
          relu_out=ptr(relu), out_absmax=ptr(amax), tmpl_split=ptr(tsplit), total_rows=rows, B=B, C=C, H=H, W=W,
          U=U, max_ht=mh, max_wt=mw, min_k=1, algo=XCORR_ALGOS["mfma"], prec=pc, stream=stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(amax.cpu().numpy(), np.abs(got).reshape(U, -1).max(1))
    assert np.array_equal(relu.cpu().numpy(), np.maximum(got, 0))
    tol = TOL if prec == "fp32" else XCORR_ONE_TERM_TOL[prec]
    tmpl_h = tmpl.cpu().numpy()
    for u in range(U):
        ht, wt, off = int(units["ht"][u]), int(units["wt"][u]), int(units["tmpl_offset"][u])
        t = tmpl_h[off:off + C * ht * wt].reshape(C, ht, wt)
        # the contract is stated against the exact correlation (float64, FFT):
        # the fp32 oracle's own sequential accumulation over h*w taps drifts by
        # up to ~1.2e-5 on constant planes (every rounding of equal products
        # biased one way), past the tolerance it is meant to check
        exact = _xcorr_exact(f[ui[u]], t, sc)
        e = normwise(got[u], exact)
        assert e <= tol, (seed, u, ht, wt, H, W, C, prec, int(kind), e, normwise(oracle.xcorr(f[ui[u]], t, sc), exact))


def _xcorr_exact(f, t, scale):
    """The correlation in float64 (scipy FFT, relative error ~1e-15 of the
    largest output): zero pad border, / (h*w), * scale; rounded to fp32."""
    from scipy.signal import fftconvolve
    C, H, W = f.shape
    h, w = t.shape[-2:]
    out = np.zeros((C, H, W), np.float64)
    for c in range(C):
        v = fftconvolve(f[c].astype(np.float64), t[c, ::-1, ::-1].astype(np.float64), mode="valid")
        out[c, h // 2:h // 2 + H - h + 1, w // 2:w // 2 + W - w + 1] = v / (h * w) * float(scale)
    return out


def _xcorr_mfma_case(H, W, C, kmax, prec):
    from tmr_amd._lib import PREC_CODES, XCORR_ALGOS, call, ptr, size, stream, xcorr
    from tmr_amd.engine import _h2d, _units_to_device
    B = 2
    f = synth.normal(90 + H + W, (B, C, H, W)) * 1.7
    shapes = [(1, 1), (3, 3), (5, 9), (7, 7), (11, 3), (13, 15), (15, 15), (17, 17), (19, 5), (21, 23),
              (25, 25), (27, 31), (31, 29), (31, 31), (9, 1), (1, 13)]
    shapes = [(min(kh, kmax, H // 2 * 2 - 1), min(kw, kmax, W // 2 * 2 - 1)) for kh, kw in shapes]
    boxes, ui = [], []
    for u, (kh, kw) in enumerate(shapes):
        boxes.append(synth.exemplar_box(kh, H, W, (5 * u) % (H - kh + 1), (7 * u) % (W - kw + 1), kw))
        ui.append(u * B // len(shapes))
    boxes = np.stack(boxes)
    units, tfl, mh, mw = host.build_units(boxes, ui, H, W, C)
    fd = cuda(f)
    tm = tmr_amd.TemplateMatching("roi_align").to(DEV)
    tmpl = torch.cat([tm.extract_template(fd[ui[u]:ui[u] + 1], torch.from_numpy(boxes[u])).reshape(-1)
                      for u in range(len(ui))])
    ud = _units_to_device(units, DEV)
    iu = _h2d(host.image_ranges(ui, B), DEV)
    U = len(ui)
    scale = torch.tensor([0.75], device=DEV)
    rows = host.tsplit_rows(units)
    tsplit = torch.empty(size("template_split", U, C, rows), device=DEV, dtype=torch.uint8)
    pc = PREC_CODES[prec]
    call("tmr_template_split", ptr(tmpl), ptr(ud), U, C, rows, pc, ptr(tsplit), stream())
    common = dict(f=ptr(fd), templates=ptr(tmpl), units=ptr(ud), img_units=ptr(iu), scale=ptr(scale),
                  tmpl_split=ptr(tsplit), total_rows=rows, B=B, C=C, H=H, W=W, U=U, max_ht=mh, max_wt=mw,
                  min_k=1, stream=stream())
    outs = {}
    for algo in ("valu", "mfma"):
        out = torch.empty((U, C, H, W), device=DEV)
        relu = torch.empty_like(out)
        amax = torch.zeros(U, device=DEV)
        xcorr(out=ptr(out), relu_out=ptr(relu), out_absmax=ptr(amax), algo=XCORR_ALGOS[algo], prec=pc, **common)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        outs[algo] = got
        # the fused per-unit max |f_TM| (the decoder's per-unit scale source)
        assert np.array_equal(amax.cpu().numpy(), np.abs(got).reshape(U, -1).max(1)), algo
        assert np.array_equal(relu.cpu().numpy(), np.maximum(got, 0)), algo
        if algo == "mfma" and prec == "bf16":
            # tmr_xcorr's bf16 plane (out_bf16): RNE bf16 of the fp32 plane, bit for bit
            o16 = torch.empty((U, C, H, W), device=DEV, dtype=torch.bfloat16)
            xcorr(out=ptr(o16), out_absmax=ptr(amax), algo=XCORR_ALGOS[algo], prec=pc, out_bf16=1, **common)
            torch.cuda.synchronize()
            assert torch.equal(o16.view(torch.int16), out.to(torch.bfloat16).view(torch.int16))
            # refused with a relu output, on the VALU kernel and on other precisions
            for bad in ((ptr(relu), XCORR_ALGOS["mfma"], pc), (None, XCORR_ALGOS["valu"], pc),
                        (None, XCORR_ALGOS["mfma"], PREC_CODES["f16"])):
                with pytest.raises(tmr_amd.TMRError):
                    xcorr(out=ptr(o16), relu_out=bad[0], algo=bad[1], prec=bad[2], out_bf16=1, **common)
            # AUTO without the split templates runs the VALU kernel (no MFMA operands): the fp32 plane
            o_auto = torch.empty((U, C, H, W), device=DEV)
            cm = dict(common, tmpl_split=None, total_rows=0)
            xcorr(out=ptr(o_auto), algo=XCORR_ALGOS["auto"], prec=pc, **cm)
            torch.cuda.synchronize()
            assert normwise(o_auto.cpu().numpy(), outs["valu"]) == 0.0
            with pytest.raises(tmr_amd.TMRError):  # MFMA without them is unsupported
                xcorr(out=ptr(o_auto), algo=XCORR_ALGOS["mfma"], prec=pc, **cm)
    tol = {"valu": TOL, "mfma": TOL if prec == "fp32" else XCORR_ONE_TERM_TOL[prec]}
    tmpl_h = tmpl.cpu().numpy()
    worst = 0.0
    for u in range(U):
        ht, wt, off = int(units["ht"][u]), int(units["wt"][u]), int(units["tmpl_offset"][u])
        t = tmpl_h[off:off + C * ht * wt].reshape(C, ht, wt)
        ref = oracle.xcorr(f[ui[u]], t, 0.75)
        for algo, got in outs.items():
            err = normwise(got[u], ref)
            assert err <= tol[algo], (algo, prec, u, ht, wt, err)
            if algo == "mfma":
                worst = max(worst, err)
            ph, pw = ht // 2, wt // 2
            if ph:
                assert (got[u][:, :ph] == 0).all() and (got[u][:, H - ph:] == 0).all()
            if pw:
                assert (got[u][:, :, :pw] == 0).all() and (got[u][:, :, W - pw:] == 0).all()
    print(f"xcorr mfma {prec} {H}x{W}: worst normwise {worst:.3e}")


def test_engine_bf16_ftm_plane_bitexact():
    """Under the bf16 contract the detect path's correlation writes f_TM as
    bf16 (tmr_xcorr out_bf16), a plane the decoder packs with
    tmr_split_xpack16: the maps are bit-identical to the fp32-plane path
    (engine.out_bf16 = False), for the shared (E = 3) and the unshared (E = 1)
    fp half, decoder kernel sizes 3 and 5."""
    cin, emb, hf = 64, 128, 32
    for k in (3, 5):
        P = synth.reference_state_dict(9, cin=cin, emb=emb, obj_bias=-0.3, k=k)
        for B, E in ((2, 3), (3, 1)):
            feats = synth.sam_features(70 + E, B, cin, hf, hf)
            ex, _ = synth.exemplar_set(71 + E, B, E, 2 * hf, 2 * hf, 3, 15)
            ui = np.repeat(np.arange(B), E)
            res = {}
            for mode in ("fp32", "plane"):
                eng = tmr_amd.TMREngine({k_: cuda(v) for k_, v in P.items()},
                                        tmr_amd.PathConfig(emb_dim=emb, precision="bf16", decoder_kernel_size=k))
                eng.xcorr_algo = "mfma"
                eng.out_bf16 = mode != "fp32"
                r = eng.forward_units(cuda(feats), ui, ex.reshape(-1, 4))
                assert eng.last_xcorr_out16 == (mode != "fp32")
                res[mode] = (r["o"].cpu().numpy(), r["b"].cpu().numpy())
            for a, b in zip(res["fp32"], res["plane"]):
                assert bits_equal(a, b), (k, B, E)
        # the module form (relu(f_TM) returned) keeps the fp32 plane
        eng.forward_units(cuda(feats), ui, ex.reshape(-1, 4), want_aux=True)
        assert not eng.last_xcorr_out16


def test_xcorr_mfma_refuses_other_widths():
    """The MFMA correlation runs W % 64 == 0 (64-column accumulator groups):
    another width is TMR_E_UNSUPPORTED under TMR_XCORR_MFMA, and the engine's
    cost model ('auto') runs the VALU kernel there."""
    C, H, W = 8, 40, 96
    f = synth.normal(6, (1, C, H, W))
    boxes = np.stack([synth.exemplar_box(k, H, W, 5, 7) for k in (5, 13)])
    P = {"matcher.scale": torch.tensor([1.0], device=DEV)}
    eng = tmr_amd.TMREngine(P, tmr_amd.PathConfig(emb_dim=C))
    eng.xcorr_algo = "mfma"
    with pytest.raises(tmr_amd.TMRError):
        eng.match(cuda(f), [0, 0], boxes)
    eng.xcorr_algo = "auto"
    out, _ = eng.match(cuda(f), [0, 0], boxes)
    assert eng.last_xcorr_algo == "valu"
    for u in range(2):
        roi, ht, wt = oracle.template_size(boxes[u], H, W)
        ref = oracle.xcorr(f[0], oracle.roi_align(f[0], roi, ht, wt), 1.0)
        assert normwise(out[u].cpu().numpy(), ref) <= TOL
    # 256 columns with a 31-row template: the band + halo + 3 over-rows exceed the
    # MFMA kernel's staging registers, so 'auto' must pick the VALU kernel, not fail
    W2 = 256
    f2 = synth.normal(16, (1, C, H, W2))
    boxes2 = np.stack([synth.exemplar_box(k, H, W2, 3, 9) for k in (31, 29)])
    out2, _ = eng.match(cuda(f2), [0, 0], boxes2)
    assert eng.last_xcorr_algo == "valu"
    for u in range(2):
        roi, ht, wt = oracle.template_size(boxes2[u], H, W2)
        ref = oracle.xcorr(f2[0], oracle.roi_align(f2[0], roi, ht, wt), 1.0)
        assert normwise(out2[u].cpu().numpy(), ref) <= TOL


def test_xcorr_mfma_squeeze_and_engine():
    """squeeze through the MFMA kernel, and TMREngine.match with xcorr_algo
    'mfma' / 'valu' / 'auto' on the scripted shape (C = 512, 128^2)."""
    C, H, W = 512, 128, 128
    f = synth.normal(5, (2, C, H, W))
    boxes = np.stack([synth.exemplar_box(k, H, W, 10 + k, 3 * k) for k in (3, 9, 15)])
    ui = [0, 0, 1]
    res = {}
    for sq in (False, True):
        P = {"matcher.scale": torch.tensor([1.25], device=DEV)}
        for algo in ("valu", "mfma", "auto"):
            eng = tmr_amd.TMREngine(P, tmr_amd.PathConfig(emb_dim=C, squeeze=sq))
            eng.xcorr_algo = algo
            out, _ = eng.match(cuda(f), ui, boxes)
            res[(sq, algo)] = out.cpu().numpy()
        for u in range(3):
            roi, ht, wt = oracle.template_size(boxes[u], H, W)
            t = oracle.roi_align(f[ui[u]], roi, ht, wt)
            ref = oracle.xcorr(f[ui[u]], t, 1.25, sq)
            for algo in ("valu", "mfma", "auto"):
                assert normwise(res[(sq, algo)][u], ref) <= TOL, (sq, algo, u)


@pytest.mark.parametrize("thr", [0.1, 0.5, 0.999, 0.9999999, 0.99999994, 1.0, 0.0, 1e-30])
def test_peaks_without_prob_match_with_prob(thr):
    """TMREngine.peaks without the probability map (detect, Get_pred_boxes)
    stages a logit well below the threshold's as -1 instead of its sigmoid:
    the candidates, their order, logits, refs and boxes are bit-identical to
    the run that writes prob -- logits straddling logit(thr) by ulps, NaN
    and +-inf logits, saturated maps, every mask shape, W of 64 / 96 / 130
    (whole-row chunks of different heights)."""
    for H, W in ((64, 64), (48, 96), (33, 130)):
        U = 6
        o = (synth.normal(811 + W, (U, 1, H, W)) * 3.0).astype(np.float32)
        if 0.0 < thr < 1.0:
            lg = np.float32(np.log(thr / (1.0 - thr)))
            away = np.where(np.arange(40) % 2, 1e9, -1e9).astype(np.float32)
            near = np.nextafter(np.full(40, lg, np.float32), away)
            o[0, 0, 5, :40] = near
            o[1, 0, 7, 3:43] = lg
            # a sweep across the band of logits whose sigmoid ROUNDS to thr (near 1 that
            # band is far wider than ulps of the logit: ADVICE r5)
            o[4, 0, 2, :64] = np.linspace(lg - 0.7, lg + 0.7, 64, dtype=np.float32)
            o[4, 0, 4, :64] = np.linspace(lg - 0.7, lg + 0.7, 64, dtype=np.float32)[::-1]
        o[2, 0, 3, 4] = np.nan
        o[2, 0, 9, 9] = np.inf
        o[2, 0, 11, 2] = -np.inf
        o[3] = 40.0  # saturated: p == 1 everywhere (ties)
        reg = (synth.normal(812 + W, (U, 4, H, W)) * 0.3).astype(np.float32)
        side = np.array([1.5, 4.0, 9.0, 1.5, 4.0, 9.0], np.float32)
        boxes = np.stack([np.full(U, 0.2, np.float32), np.full(U, 0.3, np.float32),
                          0.2 + side / W, 0.3 + side / H], 1).astype(np.float32)
        params = host.peak_params(boxes, H, W, thr)
        a = tmr_amd.TMREngine.peaks(cuda(o), cuda(reg), params, want_prob=True)
        b = tmr_amd.TMREngine.peaks(cuda(o), cuda(reg), params, want_prob=False)
        assert b[4] is None
        ca, cb = a[3].cpu().numpy(), b[3].cpu().numpy()
        assert np.array_equal(ca, cb), (H, W, thr)
        for t in range(3):
            x, y = a[t].cpu().numpy(), b[t].cpu().numpy()
            rows = x.reshape(U, H * W, -1), y.reshape(U, H * W, -1)
            for u in range(U):
                k = max(int(ca[u]), 1)
                assert bits_equal(rows[0][u, :k], rows[1][u, :k]), (H, W, thr, t, u)


def test_nms_worst_case_dense_candidates():
    """SURVEY.md §7.3.3 worst case: a centre-only adaptive kernel (exemplars
    under 2 px) with p ~ 0.5 everywhere at cls 0.1 makes EVERY pixel a
    candidate: n = E * H * W = 49,152 per image (E = 3, 128^2), two images.
    Boxes decoded from wide regressions overlap heavily.  The strip NMS
    (bounded memory, sorted by a segmented radix sort) keeps exactly the
    oracle's sequential torchvision list."""
    H = W = 128
    B, E = 2, 3
    U = B * E
    o = synth.normal(501, (U, 1, H, W)) * 0.05  # p = sigmoid(o) ~ 0.5, near-ties
    o[:, :, ::7, ::5] = 0.0  # exact ties across units
    reg = synth.normal(502, (U, 4, H, W)) * 0.4
    reg[:, 2:] += 2.3  # exp -> ~10x the exemplar size: dense overlaps
    boxes = np.array([[0.3, 0.3, 0.3 + 1.5 / W, 0.3 + 1.5 / H]] * U, np.float32)
    params = host.peak_params(boxes, H, W, 0.1)
    assert (params["mask"] == host.KERNEL_CENTER).all()
    logits, box, ref, counts, prob = tmr_amd.TMREngine.peaks(cuda(o), cuda(reg), params)
    counts_h = counts.cpu().numpy()
    assert (counts_h == H * W).all()
    unit_off = torch.arange(U, device=DEV, dtype=torch.int64) * (H * W)
    L, Bx, R, K = tmr_amd.TMREngine.nms(logits, box, ref, counts, counts_h, unit_off,
                                         np.arange(0, U + 1, E), 0.5, want_keep=True)
    lg = logits.cpu().numpy().reshape(U, H * W, 2)
    bx = box.cpu().numpy().reshape(U, H * W, 4)
    for img in range(B):
        cb = bx[img * E:(img + 1) * E].reshape(-1, 4)
        cs = lg[img * E:(img + 1) * E, :, 0].reshape(-1)
        keep = oracle.nms(cb, cs, 0.5)
        assert cb.shape[0] == 49152
        assert np.array_equal(K[img].cpu().numpy(), keep), img
        assert bits_equal(Bx[img].cpu().numpy(), cb[keep])
        assert bits_equal(L[img].cpu().numpy()[:, 0], cs[keep])


def test_detect_graph_replay_matches_eager():
    """TMREngine.detect's HIP-graph path: the second call of a launch
    signature captures the forward (projection ... peaks), later calls replay
    it with refilled host inputs.  Every call -- eager, capture, replay with
    other features, with other exemplar boxes of the same template sizes, and
    after a weight update (a new signature) -- returns exactly the eager
    engine's detections."""
    cin, emb, hf, B, E = 32, 64, 16, 2, 3
    P = synth.reference_state_dict(12, cin=cin, emb=emb, obj_bias=0.4)
    Pd = {k: cuda(v) for k, v in P.items()}
    eng = tmr_amd.TMREngine(Pd, tmr_amd.PathConfig(emb_dim=emb))
    ref = tmr_amd.TMREngine({k: v.clone() for k, v in Pd.items()}, tmr_amd.PathConfig(emb_dim=emb))
    ref.use_graphs = False
    ex0, _ = synth.exemplar_set(40, B, E, 2 * hf, 2 * hf, 3, 7)

    def shifted(ex, d):  # same template sizes, other boxes (moved only where they stay inside)
        out = ex.copy()
        ok = (out[..., 0] + d >= 0.0) & (out[..., 2] + d <= 1.0)
        out[..., 0] = np.where(ok, out[..., 0] + d, out[..., 0])
        out[..., 2] = np.where(ok, out[..., 2] + d, out[..., 2])
        return out.astype(np.float32)

    cases = [(41, ex0), (41, ex0), (42, ex0), (43, shifted(ex0, 0.01)), (44, shifted(ex0, -0.02))]
    modes = []
    for seed, ex in cases:
        feats = cuda(synth.sam_features(seed, B, cin, hf, hf))
        got = eng.detect(feats, ex, 0.5, 0.5)
        modes.append(eng.last_graph)
        want = ref.detect(feats, ex, 0.5, 0.5)
        for g_, w_ in zip(got, want):
            for a, b in zip(g_, w_):
                assert bits_equal(a.cpu().numpy(), b.cpu().numpy()), (seed, eng.last_graph)
    assert modes[0] == "eager" and modes[1] == "captured" and modes[2:] == ["replay"] * 3, \
        (modes, eng.last_graph_error)
    # the in-forward small NMS (tmr_nms_small, one sync) and its fallback to
    # tmr_nms when an image's union exceeds TMR_NMS_SMALL rows: both equal
    # the eager engine's separate NMS, through eager, capture and replay
    small = []
    for cls, h2 in ((0.9, hf), (0.9, hf), (0.9, hf), (0.0, 2 * hf), (0.0, 2 * hf), (0.0, 2 * hf), (0.5, hf)):
        feats = cuda(synth.sam_features(46, B, cin, h2, h2))
        got = eng.detect(feats, ex0, cls, 0.3)
        small.append(eng.last_nms_small)
        want = ref.detect(feats, ex0, cls, 0.3)
        for g_, w_ in zip(got, want):
            for a, b in zip(g_, w_):
                assert bits_equal(a.cpu().numpy(), b.cpu().numpy()), (cls, eng.last_graph)
    assert small[:3] == [True] * 3 and small[3:6] == [False] * 3, small
    # a weight update is a new signature: eager again, never a stale replay
    with torch.no_grad():
        eng.P["objectness_head.head.0.bias"].add_(0.1)
        ref.P["objectness_head.head.0.bias"].add_(0.1)
    feats = cuda(synth.sam_features(45, B, cin, hf, hf))
    got, want = eng.detect(feats, ex0, 0.5, 0.5), ref.detect(feats, ex0, 0.5, 0.5)
    assert eng.last_graph == "eager"
    for g_, w_ in zip(got, want):
        for a, b in zip(g_, w_):
            assert bits_equal(a.cpu().numpy(), b.cpu().numpy())
