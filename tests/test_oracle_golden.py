"""Pins the CPU oracle (oracle/) against golden vectors produced by the
reference itself (oracle/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def normwise(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).max() if b.size else 1.0
    return float(np.abs(a - b).max() / max(den, 1e-30)) if a.size else 0.0


def corner_ok(a, b):
    """Box corners: cx -/+ w/2 cancels near 0, so a 1-ulp difference in exp()
    shows up as many ulps of a small corner.  Compare in units of the ulp of the
    row's largest |coordinate| (<= 2)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    if a.size == 0:
        return True
    if not np.array_equal(np.isnan(a), np.isnan(b)):
        return False
    ok = np.isnan(b) | (a == b)  # NaN where the reference has NaN (a NaN regression), inf alike
    scale = np.spacing(np.nanmax(np.abs(np.where(np.isfinite(b), b, 0)), axis=-1, keepdims=True).astype(np.float32))
    with np.errstate(invalid="ignore"):
        return bool((ok | (np.abs(a.astype(np.float64) - b) <= 2 * scale)).all())


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


def test_xcorr_c_and_torch(golden):
    g = golden("xcorr")
    for i in range(int(g["n"])):
        C, H, W, h, w, sq = g[f"c{i}_meta"].tolist()
        f, t, ref = g[f"c{i}_f"], g[f"c{i}_t"], g[f"c{i}_out"]
        out_c = oracle.xcorr(f[0], t[0], 1.0, bool(sq))
        assert out_c.shape == ref.shape[1:]
        assert normwise(out_c, ref[0]) <= 1e-6, (i, normwise(out_c, ref[0]))
        out_t = oracle.cross_correlation_torch(torch.from_numpy(f), torch.from_numpy(t), bool(sq))
        assert normwise(out_t.numpy(), ref) <= 1e-6


def test_template_sizing_and_roi(golden):
    g = golden("template")
    f = g["f"]
    off = 0
    H, W = f.shape[-2:]
    for i, box in enumerate(g["boxes"]):
        roi, ht, wt = oracle.template_size(box, H, W)
        assert (ht, wt) == tuple(g["sizes"][i]), i
        assert np.array_equal(roi.view(np.uint32), g["rois"][i].view(np.uint32)), i
        t = oracle.roi_align(f[0], roi, ht, wt)
        n = t.size
        assert np.array_equal(t.ravel(), g["templates"][off:off + n]), i
        off += n
        pb = oracle.prototype_box(box, H, W)
        pr = oracle.prototype(f[0], pb)
        assert normwise(pr, g["protos"][i]) <= 1e-5, i


def _state(g):
    return {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}


@pytest.mark.parametrize("name", ["default", "squeeze", "prototype", "nofusion", "noboxreg",
                                  "twolayer_k5", "noupsample", "nomatcher"])
def test_forward_variants(golden, name):
    g = golden(f"forward_{name}")
    args = json.loads(str(g["args"]))
    P = _state(g)
    feats = torch.from_numpy(g["feats"])
    ex = [torch.from_numpy(e) for e in g["exemplars"]]
    os_, bs_, ftm, f0 = oracle.forward_torch(
        feats, ex, P, feature_upsample=args["feature_upsample"], fusion=args["fusion"],
        squeeze=args["squeeze"], box_reg=not args["ablation_no_box_regression"],
        template_type=args["template_type"], no_matcher=args["no_matcher"])
    assert normwise(os_[0].numpy(), g["o"]) <= 1e-5
    if "b" in g:
        assert normwise(bs_[0].numpy(), g["b"]) <= 1e-5
    else:
        assert bs_[0] is None
    assert normwise(ftm[0].numpy(), g["f_tm"]) <= 1e-5
    assert normwise(f0.numpy(), g["f0"]) <= 1e-6
    if args["feature_upsample"]:
        # the C restatement of the bilinear x2 (Appendix C) against ATen's output
        up = np.stack([oracle.upsample2x(x) for x in g["feats"]])
        assert normwise(up, g["f0"]) <= 1e-6


def _split(g, key):
    counts = g[key + "_counts"]
    arr = g[key]
    out, o = [], 0
    for c in counts:
        out.append(arr[o:o + c]); o += c
    return out


@pytest.mark.parametrize("name", ["pred_boxes", "pred_boxes_nonfinite"])
def test_pred_boxes(golden, name):
    """Every candidate bit-exact vs the reference's Get_pred_boxes; the
    _nonfinite fixture pins NaN / +-inf maps (torch.max's NaN propagation
    through the masked 3x3 window, TM_utils.py:253,359)."""
    g = golden(name)
    max_ulp = 0
    for i in range(int(g["n"])):
        meta = json.loads(str(g[f"c{i}_meta"]))
        probs, reg, ex = g[f"c{i}_prob"], g[f"c{i}_reg"], g[f"c{i}_ex"]
        L, Bx, R = oracle.get_pred_boxes_prob(
            list(probs), list(reg) if meta["box_reg"] else None, [e[None] for e in ex],
            meta["thr"], meta["box_reg"], meta["ab_b"], meta["ab_c"])
        gL, gB, gR = _split(g, f"c{i}_logits"), _split(g, f"c{i}_boxes"), _split(g, f"c{i}_refs")
        for b in range(len(L)):
            assert L[b].shape == gL[b].shape, (i, b, meta)
            assert np.array_equal(L[b], gL[b]), (i, b)
            assert np.array_equal(R[b], gR[b]), (i, b)
            # the decode with the reference's own exp (torch.exp on CPU = MKL
            # vsExp): bit-exact; with a correctly rounded exp instead, ~0.2%
            # of the corners move (1 ulp of exp, cancellation in cx -/+ w/2)
            assert np.array_equal(Bx[b].view(np.uint32), gB[b].view(np.uint32)), (i, b, meta)
            _, Bc, _ = oracle.get_pred_boxes_prob(
                [probs[b]], [reg[b]] if meta["box_reg"] else None, [ex[b][None]], meta["thr"],
                meta["box_reg"], meta["ab_b"], meta["ab_c"], exp_mode="cr")
            d = ulp_diff(Bc[0], gB[b])
            max_ulp = max(max_ulp, int(d.max()) if d.size else 0)
            assert corner_ok(Bc[0], gB[b]), (i, b, meta)
    print("correctly rounded exp instead: max corner ulp diff vs reference:", max_ulp)


@pytest.mark.parametrize("name", ["nms", "nms_nonfinite"])
def test_nms(golden, name):
    """Keep lists vs the reference's NMS (through the nms transcription; the
    _nonfinite fixture: NaN scores first as torch.sort(descending) puts them,
    +-inf, -0.0 == +0.0, NaN / inf coordinates)."""
    g = golden(name)
    for i in range(int(g["n"])):
        keep = oracle.nms(g[f"c{i}_boxes"], g[f"c{i}_scores"], float(g[f"c{i}_thr"]))
        assert np.array_equal(keep, g[f"c{i}_keep"]), i
        if f"c{i}_kept_boxes" in g and g[f"c{i}_boxes"].shape[0]:
            assert np.array_equal(g[f"c{i}_boxes"][keep], g[f"c{i}_kept_boxes"], equal_nan=True), i


def test_caller_sequence(golden):
    g = golden("caller")
    P = _state(g)
    feats = torch.from_numpy(g["feats"])
    ex = g["exemplars"]
    for thr, iou in ((0.1, 0.5), (0.5, 0.15), (0.7, 0.5)):
        L, Bx, R = [], [], []
        for e in range(ex.shape[1]):
            exemplar = [torch.from_numpy(ex[0, e:e + 1])]
            o, b, _, _ = oracle.forward_torch(feats, exemplar, P)
            prob = o[0][0].sigmoid().squeeze(0).numpy()
            l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [b[0][0].numpy()], exemplar, thr)
            L.append(l_[0]); Bx.append(b_[0]); R.append(r_[0])
        L, Bx, R = oracle.nms_lists([np.concatenate(L)], [np.concatenate(Bx)], [np.concatenate(R)],
                                    iou)
        tag = f"t{int(thr * 100)}_i{int(iou * 100)}"
        assert L[0].shape == g[f"{tag}_logits"].shape
        assert np.array_equal(L[0], g[f"{tag}_logits"])
        assert np.array_equal(R[0], g[f"{tag}_refs"])
        assert np.array_equal(Bx[0].view(np.uint32), g[f"{tag}_boxes"].view(np.uint32))


def test_reference_exp_characterised():
    """The reference decode's torch.exp (ATen CPU fp32 -> MKL vsExp) is a
    function of the value alone (no position / length dependence) and within
    one ulp of the correctly rounded exp.  On the host the table was recorded
    on (the golden vectors' host), correctly rounded + the table's one-ulp
    moves (oracle.expf "reference") reproduce torch.exp exactly; MKL takes
    other paths on other CPUs (exp_table.py), where only the recorded-table
    restatement -- host independent -- is the golden vectors' exp."""
    from tmr_amd import exp_table
    raw = exp_table.read()
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.normal(0, 3, 300000), rng.normal(0, 1e-3, 100000),
                        -np.abs(rng.normal(0, 1e-6, 100000))]).astype(np.float32)
    t = torch.exp(torch.from_numpy(x)).numpy()
    perm = rng.permutation(x.size)
    assert np.array_equal(torch.exp(torch.from_numpy(x[perm])).numpy().view(np.uint32), t[perm].view(np.uint32))
    for n in (1, 7, 17, 33):
        assert np.array_equal(torch.exp(torch.from_numpy(x[:n])).numpy().view(np.uint32), t[:n].view(np.uint32))
    cr = oracle.expf(x, "cr")
    assert np.abs(t.view(np.int32).astype(np.int64) - cr.view(np.int32)).max() <= 1
    ref = oracle.expf(x, "reference")
    assert np.abs(ref.view(np.int32).astype(np.int64) - cr.view(np.int32)).max() <= 1
    assert (ref != cr).any()
    if exp_table.recorded_cpu(raw) == exp_table.host_cpu():
        assert np.array_equal(ref.view(np.uint32), t.view(np.uint32))


def test_reference_exp_table_pinned(tmp_path, monkeypatch):
    """The reference-exp table is the golden host's: its payload SHA-256 is
    pinned, this host's torch.exp matches the committed golden sample on the
    golden host, a different table is refused by read(), a table differing
    only in its informational header strings is accepted, and
    generation refuses a host whose torch.exp differs from the golden host's."""
    from tmr_amd import exp_table
    from tmr_amd._lib import TMRError
    raw = exp_table.read()
    assert exp_table.payload_sha256(raw) == exp_table.GOLDEN_PAYLOAD_SHA256
    assert exp_table.recorded_cpu(raw) == exp_table.GOLDEN_CPU
    ok, bad, n = exp_table.host_matches_golden()
    if exp_table.host_cpu() == exp_table.GOLDEN_CPU:
        assert ok, (bad, n)
    # the sample's recorded half really exercises the table
    with np.load(exp_table.SAMPLE, allow_pickle=False) as z:
        x, y = z["x"], z["y"]
    hit = exp_table.lookup_host(x.view(np.float32), raw)
    assert 8000 <= int(hit.sum()) <= 8192 + 200
    cr = np.exp(x.view(np.float32).astype(np.float64)).astype(np.float32).view(np.uint32)
    assert np.array_equal(hit, y != cr)  # recorded <=> the golden exp is not correctly rounded
    # a corrupted copy is refused
    bad_copy = tmp_path / "exp_ref.bin"
    b = bytearray(open(exp_table.PATH, "rb").read())
    b[HEADER_FLIP] ^= 1
    bad_copy.write_bytes(bytes(b))
    with pytest.raises(TMRError, match="sha256"):
        exp_table.read(str(bad_copy))
    # another torch build / CPU name in the header only: accepted
    other = tmp_path / "other_header.bin"
    b = bytearray(open(exp_table.PATH, "rb").read())
    b[24:56] = b"9.9.9+other".ljust(32, b"\0")
    b[56:120] = b"Some Other CPU".ljust(64, b"\0")
    other.write_bytes(bytes(b))
    assert exp_table.payload_sha256(exp_table.read(str(other))) == exp_table.GOLDEN_PAYLOAD_SHA256
    # another host's exp: generation refuses before writing anything
    monkeypatch.setattr(exp_table, "host_matches_golden", lambda sample=None: (False, 17, 16384))
    out = tmp_path / "gen.bin"
    with pytest.raises(TMRError, match="differs from the golden host"):
        exp_table.generate(str(out))
    assert not out.exists()


def test_reference_exp_table_from_committed_blob(tmp_path):
    """the table a clean checkout builds.  The compact form as
    COMMITTED at HEAD (git show, not the working tree) expands -- with no use
    of this host's torch.exp -- to the pinned payload, byte-identical to the
    golden host's table; a damaged blob is refused."""
    import subprocess
    from tmr_amd import exp_table
    from tmr_amd._lib import TMRError
    rel = os.path.relpath(exp_table.BLOB, REPO)
    try:
        blob = subprocess.run(["git", "-C", REPO, "show", f"HEAD:{rel}"], check=True,
                              capture_output=True).stdout
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("not a git checkout")
    src = tmp_path / "exp_ref.rc"
    src.write_bytes(blob)
    out = tmp_path / "exp_ref.bin"
    assert exp_table.expand(str(src), str(out)) == exp_table.GOLDEN_COUNT
    assert exp_table.payload_sha256(np.fromfile(out, np.uint8)) == exp_table.GOLDEN_PAYLOAD_SHA256
    assert exp_table.sha256(str(out)) == exp_table.GOLDEN_FILE_SHA256
    bad = bytearray(blob)
    bad[len(bad) // 2] ^= 0x10
    src.write_bytes(bytes(bad))
    with pytest.raises(TMRError):
        exp_table.expand(str(src), str(tmp_path / "bad.bin"))
    assert not (tmp_path / "bad.bin").exists()


HEADER_FLIP = 128 + 4 * 40000  # a byte inside the offsets block


def test_reference_exp_table_ensure_rebuilds_damaged(tmp_path):
    """build()'s table step (exp_table.ensure): a present golden table is
    kept, a damaged or missing one is re-expanded from the committed blob."""
    from tmr_amd import exp_table
    p = tmp_path / "exp_ref.bin"
    assert exp_table.ensure(str(p)) == "expanded"
    assert exp_table.ensure(str(p)) == "verified"
    b = bytearray(p.read_bytes())
    b[HEADER_FLIP] ^= 4
    p.write_bytes(bytes(b))
    assert exp_table.ensure(str(p)) == "expanded"
    assert exp_table.payload_sha256(np.fromfile(p, np.uint8)) == exp_table.GOLDEN_PAYLOAD_SHA256
