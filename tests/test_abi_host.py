"""CPU-only: the C-ABI library loads and exports every symbol include/tmr.h
declares; host-side descriptor arithmetic matches the oracle bit for bit."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import oracle
import tmr_amd
from tmr_amd import _lib, host, synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "tmr.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tmr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    syms = header_symbols()
    assert len(syms) >= 14
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table out of sync with tmr.h"
    L = tmr_amd.load()
    assert L.tmr_version() == 3
    # ABI 3: one correlation entry point, one sizing query, one
    # split conv entry point -- at most ~25 symbols
    assert len(syms) <= 25, syms
    assert L.tmr_strerror(0) == b"ok"
    assert b"invalid" in L.tmr_strerror(-1)


def test_struct_layouts():
    assert _lib.UNIT_DTYPE.itemsize == 64
    assert _lib.PEAK_DTYPE.itemsize == 24


def _size(kind, *d):
    return int(tmr_amd.load().tmr_size(_lib.SIZE_KINDS[kind], *(list(d) + [0] * (6 - len(d)))))


def test_size_queries_no_gpu():
    assert _size("heads_partials", 2048, 3, 8, 8) == 32 * 5 * 3 * 64  # 64-wide tiles
    assert _size("nms_work", 10, 4, 5, 3) > 10 * 40
    # linear in the candidates (the binned NMS keeps no n^2 IoU matrix): at most
    # 640 B per candidate (a 128-entry suppressor list is 512 of them) plus a
    # fixed part, 64 images x 49,152 candidates
    big = _size("nms_work", 64 * 49152, 64 * 768, 49152, 64)
    assert big < 64 * 49152 * 640 + (16 << 20)
    half = _size("nms_work", 32 * 49152, 32 * 768, 49152, 32)
    assert abs(big - 2 * half) < (4 << 20)
    # the documented worst case (include/tmr.h): one image of 589,824 candidates
    assert _size("nms_work", 589824, 589824 // 64, 589824, 1) < 0.4e9
    assert _size("template_split", 3, 512, 45) == 512 * 45 * 2 * 1024 + 4 * 3 * 512
    assert _size("stats_work", 4) > 0
    assert tmr_amd.load().tmr_size(99, 1, 1, 1, 1, 1, 1) == -1  # unknown kind
    assert _size("acc", 1 << 40, 8, 8, 8) == -1  # dimensions past int range


def test_split_size_queries_no_gpu():
    """Byte sizes of the split-kernel records (include/tmr.h): activations
    padded to whole 16x32 tiles plus the ks halo, one 64-B record per pixel per
    32-channel chunk and half (fp32 3-term: hi and lo halves); weights
    [ks^2][chunks][ceil(N/128)*128][128 B (wh, wl) | 64 B]."""
    assert _size("xpack", 2, 512, 128, 128, 3, 0) == 2 * 32 * 130 * 130 * 64
    assert _size("xpack", 2, 512, 128, 128, 3, 1) == 2 * 16 * 130 * 130 * 64
    assert _size("xpack", 1, 257, 17, 33, 1, 0) == 1 * 9 * 2 * 32 * 64 * 64
    assert _size("xpack", 1, 8, 8, 8, 4, 0) == -1   # even kernel
    assert _size("xpack", 1, 8, 8, 8, 3, 5) == -1   # unknown precision
    assert _size("wpack", 2048, 257, 512, 3, 0) == 9 * (9 + 16) * 2048 * 128
    assert _size("wpack", 100, 0, 40, 5, 2) == 25 * 2 * 128 * 64
    assert _size("wpack", 8, 0, 0, 3, 0) == -1


def test_invalid_arguments_return_codes():
    L = tmr_amd.load()
    assert L.tmr_heads_reduce(None, 8, 128, 1, 4, 4, None, None, None, None) == -1
    assert L.tmr_upsample2x(None, 1, 4, 4, None, None) == -1
    # the compact reference-exp table: a malformed blob is refused
    junk = np.zeros(64, np.uint8)
    assert L.tmr_exp_table_decode(junk.ctypes.data, junk.size, None, 0) == -1
    assert L.tmr_xcorr(None, None) == -1
    args = _lib.XcorrArgs()
    args.B = args.C = args.H = args.W = args.U = args.max_ht = args.max_wt = 1
    assert L.tmr_xcorr(ctypes.byref(args), None) == -1  # NULL tensors
    assert ctypes.sizeof(_lib.XcorrArgs) == 10 * 8 + 8 + 12 * 4  # tmr_xcorr_args_t
    assert L.tmr_nms(*([None] * 8), 0, 0, 0, 0, 0.5, *([None] * 7)) == -1
    # split conv: bad precision / kernel size / missing scale sources never launch
    assert L.tmr_split_conv(None, 0, None, None, 8, 1, 8, 8, 3, 9, None, None, None, None, 8, 0,
                            None, None, None, 0, None) == -1
    assert L.tmr_split_conv(None, 0, None, None, 8, 1, 8, 8, 2, 0, None, None, None, None, 8, 1,
                            None, None, None, 0, None) == -1
    assert _size("acc", 2, 2048, 128, 128) == 2 * 2048 * 128 * 128
    assert _size("acc", 1, 100, 17, 33) == 128 * 32 * 64
    assert L.tmr_split_xpack(None, 1, 8, 8, 8, 0, 3, 0, None, 0, None, None) == -1
    buf8 = np.zeros(8, np.float32)
    assert L.tmr_split_xpack(buf8.ctypes.data, 1, 8, 8, 8, 4, 3, 0, buf8.ctypes.data, 0, buf8.ctypes.data,
                             None) == -1  # unknown `up` bit
    # per-sample scale sources (ABI 2): missing pointers / empty batches never launch
    assert L.tmr_absmax_rows(None, 2, 4, 0, None, None) == -1
    assert L.tmr_absmax_rows(None, 0, 4, 0, None, None) == -1
    assert L.tmr_scale_merge(None, None, None, 2, 3, None, None, None) == -1
    # masked maxpool: an empty selection (torch.max rejects it) or bits past the 3x3 window
    assert L.tmr_maxpool3x3(None, 1, 4, 4, 0, None, None) == -1
    assert L.tmr_maxpool3x3(None, 1, 4, 4, 1 << 9, None, None) == -1
    assert L.tmr_maxpool3x3(None, 0, 4, 4, 0x1ff, None, None) == 0  # empty input: nothing to launch
    # peaks: prob is required (scratch with TMR_PEAKS_PROB_SCRATCH); unknown flag bits are refused
    buf = np.zeros(16, np.float32)
    a = buf.ctypes.data
    assert L.tmr_peaks_decode(a, 0, None, 1, 2, 2, a, None, a, a, a, a, None, None) == -1
    assert L.tmr_peaks_decode(a, 4, None, 1, 2, 2, a, a, a, a, a, a, None, None) == -1
    # NMS: an image beyond the greedy wave's LDS bitmap (655,360 candidates) is refused, not truncated
    big = 700_000
    assert L.tmr_nms(a, a, a, a, a, a, a, a, 1, big, big, (big + 63) // 64, 0.5, a, a, a, None, a, a,
                     None) == -1


def test_tm_utils_host_helpers():
    import torch
    assert tmr_amd.calc_area([1.0, 2.0, 4.0, 7.0]) == 15.0
    x = np.array([[1.0, 3.0], [2.0, 5.0]], np.float32)
    np.testing.assert_array_equal(tmr_amd.map_normalization(x), (x - 1.0) / (4.0 + 1e-14))
    t = tmr_amd.map_normalization(torch.from_numpy(x))
    assert torch.equal(t, (torch.from_numpy(x) - 1.0) / (4.0 + 1e-14))
    with pytest.raises(tmr_amd.TMRError):  # GPU only, no CPU fallback
        tmr_amd.custom_shape_3x3_maxpool2d(torch.zeros(1, 1, 4, 4), [[1] * 3] * 3)


def test_gpu_only_guard():
    import torch
    with pytest.raises(tmr_amd.TMRError):
        tmr_amd.Decoder_model(8)(torch.zeros(1, 8, 4, 4))


def _rand_boxes(seed, n):
    u = synth.uniform(seed, 4 * n).reshape(n, 4).astype(np.float32)
    x1 = u[:, 0] * 1.2 - 0.1
    y1 = u[:, 1] * 1.2 - 0.1
    return np.stack([x1, y1, x1 + 0.005 + u[:, 2] * 0.5, y1 + 0.005 + u[:, 3] * 0.5], 1).astype(np.float32)


@pytest.mark.parametrize("HW", [(32, 32), (128, 128), (192, 192), (24, 40)])
def test_template_sizing_matches_oracle(HW):
    H, W = HW
    for box in _rand_boxes(H * 7 + W, 400):
        try:
            roi, ht, wt = host.template_size(box, H, W)
        except ValueError:
            with pytest.raises(ValueError):
                oracle.template_size(box, H, W)
            continue
        oroi, oht, owt = oracle.template_size(box, H, W)
        assert (ht, wt) == (oht, owt)
        assert np.array_equal(roi.view(np.uint32), oroi.view(np.uint32))
        assert np.array_equal(host.prototype_box(box, H, W), oracle.prototype_box(box, H, W))


def test_template_sizing_golden(golden):
    g = golden("template")
    H, W = g["f"].shape[-2:]
    for i, box in enumerate(g["boxes"]):
        roi, ht, wt = host.template_size(box, H, W)
        assert (ht, wt) == tuple(g["sizes"][i])
        assert np.array_equal(roi.view(np.uint32), g["rois"][i].view(np.uint32))


def test_synthetic_boxes_give_requested_size():
    for k in range(1, 32, 2):
        for H in (64, 128, 192):
            box = synth.exemplar_box(k, H, H, 5, 7)
            _, ht, wt = host.template_size(box, H, H)
            assert ht == k and wt == k


@pytest.mark.parametrize("HW", [(128, 128), (24, 32), (192, 192)])
def test_peak_params_match_oracle(HW):
    H, W = HW
    boxes = _rand_boxes(5, 300)
    # include the exact kernel boundaries 2/H and 3/H
    extra = np.array([[0.1, 0.1, 0.1 + 3.0 / W, 0.1 + 3.0 / H], [0.1, 0.1, 0.1 + 2.0 / W, 0.1 + 2.0 / H],
                      [0.2, 0.2, 0.2 + 1.0 / W, 0.2 + 2.5 / H], [0, 0, 1, 1], [-1, -1, 0, 0]], np.float32)
    boxes = np.concatenate([boxes, extra])
    for ab_b in (False, True):
        P = host.peak_params(boxes, H, W, 0.7, True, ab_b, False)
        for u, box in enumerate(boxes):
            s = oracle.exemplar_scalars(box, ab_b)
            m = oracle.adaptive_kernel(s[0], s[1], H, W).reshape(9)
            mask = sum(int(v) << i for i, v in enumerate(m))
            assert P["mask"][u] == mask
            assert P["scale_w"][u] == s[2] and P["scale_h"][u] == s[3]
            assert P["thr"][u] == np.float32(0.7)


def test_adaptive_kernel_api():
    assert tmr_amd.adaptive_kernel_generater([0.5, 0.5], [128, 128]) == [[1, 1, 1]] * 3
    assert tmr_amd.adaptive_kernel_generater([0.001, 0.001], [128, 128]) == [[0, 0, 0], [0, 1, 0], [0, 0, 0]]
    assert tmr_amd.adaptive_kernel_generater([0.001, 0.5], [128, 128]) == [[0, 1, 0]] * 3
    assert tmr_amd.adaptive_kernel_generater([0.5, 0.001], [128, 128]) == [[0, 0, 0], [1, 1, 1], [0, 0, 0]]
    assert tmr_amd.adaptive_kernel_generater([2.5 / 128, 2.5 / 128], [128, 128]) == \
        [[0, 1, 0], [1, 1, 1], [0, 1, 0]]


def test_nms_offsets_dummy_rule():
    counts = np.array([3, 0, 5, 0, 0, 2])
    seg = np.array([0, 3, 6])
    cand_off, nb_off, mx = host.nms_offsets(counts, seg)
    assert cand_off.tolist() == [0, 9, 13]  # 3+1+5, 1+1+2
    assert mx == 9
    assert nb_off.tolist() == [0, 1, 2]  # prefix sums of ceil(n/64)


def test_state_dict_keys_match_reference(golden):
    from types import SimpleNamespace
    import torch

    class BB(torch.nn.Module):
        num_channels = 16

        def forward(self, x):
            return x

    for name in ["default", "squeeze", "nofusion", "noboxreg", "twolayer_k5", "nomatcher"]:
        g = golden(f"forward_{name}")
        import json
        args = SimpleNamespace(**json.loads(str(g["args"])))
        m = tmr_amd.matching_net(BB(), args)
        ref_keys = sorted(k[3:] for k in g if k.startswith("sd."))
        assert sorted(m.state_dict().keys()) == ref_keys, name
        sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
        m.load_state_dict(sd, strict=True)


def test_build_model_reference_signature(golden):
    """build_model(args) with the reference's one-argument signature
    (models/__init__.py:4-10, trainer.py:21): the backbone comes from
    args.backbone through the registry; the Lightning 'model.' prefix loads."""
    import json
    from types import SimpleNamespace
    import torch

    g = golden("forward_default")
    a = json.loads(str(g["args"]))
    a.update(backbone="features", num_channels=g["feats"].shape[1])
    m = tmr_amd.build_model(SimpleNamespace(**a))
    assert isinstance(m.encoder.backbone, tmr_amd.FeatureInput)
    ref_keys = sorted(k[3:] for k in g if k.startswith("sd."))
    assert sorted(m.state_dict().keys()) == ref_keys

    class Lit(torch.nn.Module):  # Matching_Trainer holds the net as self.model
        def __init__(self, net):
            super().__init__()
            self.model = net

    sd = {"model." + k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    Lit(m).load_state_dict(sd, strict=True)

    # a registered stock-PyTorch encoder under a reference backbone name
    class FakeSam(torch.nn.Module):
        num_channels = 16

        def forward(self, x):
            return x

    tmr_amd.register_backbone("sam", lambda args: FakeSam())
    try:
        m2 = tmr_amd.build_model(SimpleNamespace(**dict(a, backbone="sam")))
        assert isinstance(m2.encoder.backbone, FakeSam)
    finally:
        tmr_amd.unregister_backbone("sam")
    with pytest.raises(tmr_amd.TMRError, match="not registered"):
        tmr_amd.build_model(SimpleNamespace(**dict(a, backbone="sam")))


def test_template_matching_members():
    """The reference's public members (template_matching.py:16-23)."""
    m = tmr_amd.TemplateMatching("roi_align")
    assert m.extract_function == m.extract_template
    assert m.matching_algorithm == m.cross_correlation
    assert tmr_amd.TemplateMatching("prototype").extract_function.__name__ == "extract_prototype"
    assert [k for k, _ in m.named_parameters()] == ["scale"]
    with pytest.raises(KeyError):
        tmr_amd.TemplateMatching("nope")
    assert m._native()
    m.matching_algorithm = lambda f, t: f
    assert not m._native()  # a replaced member routes through the reference loop


def test_xcorr_cost_table_committed_crossovers(tmp_path):
    """the live correlation cost model is the committed rocprof
    sweep (xcorr_cost.json), with the crossovers DESIGN.md §4.3 documents
    (single-size launches, round-6 sweep: 128^2 E=3 fp32 from k=7, one-term
    from k=5; 192^2 E=16 fp32 from k=7, one-term at every k); a malformed or incomplete
    table raises instead of silently moving them."""
    import json
    from tmr_amd import engine as e
    assert "xcorr_crossover.json" in e.XCORR_COST_SOURCE

    def first_mfma(upi, one):
        return min(k for k in range(1, 32, 2)
                   if e.xcorr_choice(np.full(8, k), np.full(8, k), upi, True, one) == "mfma")
    assert first_mfma(3, False) == 7 and first_mfma(3, True) == 5
    assert first_mfma(16, False) == 7 and first_mfma(16, True) == 1
    bad = tmp_path / "bad.json"
    bad.write_text("{not json")
    with pytest.raises(tmr_amd.TMRError, match="malformed"):
        e._load_xcorr_cost(str(bad))
    d = json.load(open(e._COST_JSON))
    d["regimes"].pop("r192_e16_bf16")
    part = tmp_path / "part.json"
    part.write_text(json.dumps(d))
    with pytest.raises(tmr_amd.TMRError, match="lacks"):
        e._load_xcorr_cost(str(part))
    assert e._load_xcorr_cost(str(tmp_path / "absent.json")) is None


def test_xcorr_cost_table_matches_kernel_sources():
    """the committed cost table (xcorr_cost.json) and its
    counter record (profiles/xcorr_crossover.json) were swept on the
    correlation kernel sources of this tree (buildinfo digest of xcorr.hip,
    tmr_common.h, Makefile): a kernel edit without re-running
    profiles/gpu_xcorr_sweep.sh turns this red, so the crossover can never
    be priced on a kernel that no longer exists."""
    import json
    from tmr_amd import buildinfo
    from tmr_amd import engine as e
    want = buildinfo.source_digest("xcorr")
    cost = json.load(open(e._COST_JSON))
    rec = json.load(open(os.path.join(REPO, "profiles", "xcorr_crossover.json")))
    assert cost.get("source_digest") == want, "xcorr_cost.json is from other sources: re-run gpu_xcorr_sweep.sh"
    assert rec.get("source_digest") == want


def test_build_units_vectorised_matches_scalar():
    """host.build_units computes the ROI sizing vectorised: the same fp32
    operations per unit as the scalar host.template_size (the reference's
    0-d tensor math), incl. boxes on the clamp edges and NaN coordinates."""
    H, W, C = 128, 96, 16
    boxes = _rand_boxes(77, 500)
    boxes = boxes[[i for i, b in enumerate(boxes) if _sizes_ok(b, H, W)]]
    extra = np.array([[0, 0, 1, 1], [0.5, 0.5, 0.5 + 3.0 / W, 0.5 + 3.0 / H], [-0.2, 0.1, 0.3, 1.4],
                      [np.nan, 0.2, 0.4, 0.6]], np.float32)
    extra = extra[[i for i, b in enumerate(extra) if _sizes_ok(b, H, W)]]
    boxes = np.concatenate([boxes, extra]).astype(np.float32)
    ui = np.sort(np.arange(len(boxes)) % 7)
    units, tfl, mh, mw = host.build_units(boxes, ui, H, W, C)
    off = rows = 0
    for u, b in enumerate(boxes):
        roi, ht, wt = host.template_size(b, H, W)
        assert (units["ht"][u], units["wt"][u]) == (ht, wt)
        assert np.array_equal(units["roi"][u].view(np.uint32), roi.view(np.uint32))
        assert units["tmpl_offset"][u] == off and units["row_offset"][u] == rows
        assert units["pad_"][u] == 0
        off += C * ht * wt
        rows += host.tsplit_windows(ht, wt)
    assert tfl == off and mh == units["ht"].max() and mw == units["wt"].max()
    with pytest.raises(ValueError):
        host.build_units(np.array([[0.5, 0.5, 0.5, 0.5]], np.float32), [0], H, W, C)
    # up to host.SMALL_UNITS units the builder runs per unit: the same records
    assert len(boxes) > host.SMALL_UNITS
    u0 = 0
    for n in list(range(1, host.SMALL_UNITS + 1)) * 8:
        if u0 + n > len(boxes):
            break
        small, tfl_s, mh_s, mw_s = host.build_units(boxes[u0:u0 + n], ui[u0:u0 + n], H, W, C)
        ref = units[u0:u0 + n].copy()
        ref["tmpl_offset"] -= ref["tmpl_offset"][0]
        ref["row_offset"] -= ref["row_offset"][0]
        for f in small.dtype.names:  # field-wise (a structured copy leaves the padding undefined)
            a, b = np.ascontiguousarray(small[f]), np.ascontiguousarray(ref[f])
            assert a.tobytes() == b.tobytes(), (u0, n, f)
        assert (mh_s, mw_s) == (max(1, ref["ht"].max()), max(1, ref["wt"].max()))
        assert tfl_s == int((C * ref["ht"].astype(np.int64) * ref["wt"]).sum())
        u0 += n
    with pytest.raises(ValueError):
        host.build_units(np.array([[0.5, 0.5, 0.5, 0.5]] * (host.SMALL_UNITS + 1), np.float32),
                         [0] * (host.SMALL_UNITS + 1), H, W, C)


def _sizes_ok(b, H, W):
    try:
        host.template_size(b, H, W)
        return True
    except ValueError:
        return False


def test_image_ranges_small_and_vector_forms_agree():
    """host.image_ranges runs per unit up to host.SMALL_UNITS units and
    vectorised above: the same [B+1] ranges, the same refusals."""
    rng = np.random.default_rng(5)
    for U in list(range(0, 2 * host.SMALL_UNITS + 2)):
        B = int(rng.integers(1, 6))
        ui = np.sort(rng.integers(0, B, U))
        want = np.zeros(B + 1, np.int64)
        for i in ui:
            want[i + 1:] += 1
        got = host.image_ranges(ui, B)
        assert got.dtype == np.int32 and np.array_equal(got, want), (U, B)
    for bad in ([1, 0], [0, 3], [-1, 0]):
        for pad in (0, host.SMALL_UNITS):
            with pytest.raises(ValueError):
                host.image_ranges([0] * pad + bad if bad[0] >= 0 else bad + [0] * pad, 3)


def test_clone_outputs_groups_views_of_one_buffer():
    """engine._clone_outputs (a replayed graph's static outputs copied out):
    contiguous views of one storage (o, b) come back as views of ONE fresh
    copy with the same values; other tensors are cloned; `fp` is kept."""
    import torch
    from tmr_amd.engine import _clone_outputs
    ob = torch.arange(50.0)
    o, b = ob[:10].view(2, 1, 5), ob[10:].view(2, 4, 5)
    f = torch.arange(7.0)
    r = _clone_outputs({"o": o, "b": b, "f0": f, "fp": f, "n": 3})
    assert torch.equal(r["o"], o) and torch.equal(r["b"], b) and torch.equal(r["f0"], f)
    assert r["fp"] is f and r["n"] == 3
    assert r["o"].untyped_storage().data_ptr() == r["b"].untyped_storage().data_ptr()
    assert r["o"].untyped_storage().data_ptr() != ob.untyped_storage().data_ptr()
    assert r["f0"].untyped_storage().data_ptr() != f.untyped_storage().data_ptr()
    ob.zero_()
    assert float(r["b"].sum()) == float(sum(range(10, 50)))
    nc = torch.arange(12.0).view(3, 4)[:, :2]  # non-contiguous views are cloned one by one
    r = _clone_outputs({"a": nc, "b": nc.t()})
    assert torch.equal(r["a"], nc) and torch.equal(r["b"], nc.t())


def test_graph_book_bounded_and_failures_remembered():
    """TMREngine's graph bookkeeping: a signature is captured on
    its second sighting; the seen-counts and the failure set are bounded
    LRUs (varied exemplar sizes make a new signature almost every batch);
    a failed capture is remembered, so that signature stays eager without
    re-trying the capture; graphs are an LRU of GRAPH_CACHE."""
    from tmr_amd.engine import TMREngine, _GraphBook
    b = _GraphBook(cap=2, seen_cap=4)
    assert not b.want_capture("a") and b.want_capture("a")
    b.put("a", "graph-a")
    assert b.get("a") == "graph-a" and "a" not in b.seen
    # the seen-counts stay bounded under a stream of one-off signatures
    for i in range(100):
        assert not b.want_capture(("once", i))
    assert len(b.seen) == 4
    # a failed capture: never retried
    assert not b.want_capture("bad") and b.want_capture("bad")
    b.put("bad", None)
    assert all(not b.want_capture("bad") for _ in range(5)) and b.get("bad") is None
    for i in range(10):
        b.put(("bad", i), None)
    assert len(b.failed) == 4
    # graphs: LRU of cap, a hit refreshes its entry
    b.put("b", "graph-b")
    assert b.get("a") == "graph-a"
    b.put("c", "graph-c")
    assert b.get("b") is None and b.get("a") == "graph-a" and b.get("c") == "graph-c"
    b.clear()
    assert not (b.graphs or b.seen or b.failed)
    assert TMREngine.GRAPH_CACHE >= 1


def test_heads_image_major_only_for_few_units_per_image():
    """The heads launch runs image-major (an image's units innermost) up to
    HEADS_IMAGE_MAJOR_MAX units per image (config B's 3: faster; config E's
    16: 1.1% slower, profiles/archive/r05/r05t), and only for units in image order."""
    from tmr_amd import engine
    upi = engine.TMREngine._units_per_image
    assert engine.HEADS_IMAGE_MAJOR_MAX == 4
    assert upi(np.repeat(np.arange(64), 3), 64) == 3
    assert upi(np.repeat(np.arange(8), 16), 8) == 1
    assert upi(np.arange(64), 64) == 1                    # one unit per image
    assert upi(np.array([0, 1, 0, 1, 0, 1]), 2) == 1      # not in image order


def test_graph_param_key_follows_the_parameter_dict():
    """The graph signature's parameter part (TMREngine._param_key): name
    order cached, but versions, replaced tensors, added and swapped keys all
    show in the key (a stale key would replay a graph on old weights)."""
    P = {"b": torch.zeros(2), "a": torch.ones(3)}
    e = tmr_amd.TMREngine(P, tmr_amd.PathConfig())
    k1 = e._param_key()
    assert [x[0] for x in k1] == ["a", "b"]
    P["a"].add_(1)
    assert e._param_key() != k1                       # in-place update: new version
    P["a"] = torch.ones(3)
    assert e._param_key()[0][1] == P["a"].data_ptr()  # replaced tensor
    del P["b"]
    P["c"] = torch.zeros(1)
    assert [x[0] for x in e._param_key()] == ["a", "c"]  # same count, other key
    P["d"] = torch.zeros(1)
    assert [x[0] for x in e._param_key()] == ["a", "c", "d"]



def test_toeplitz_table_matches_window_count():
    """profiles/mfma_shapes/toeplitz.py (the round-6 shape study's useful-rate
    table) prices the 2-D window form with the same window count the kernel
    and the template split use (host.tsplit_windows)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "toeplitz", os.path.join(REPO, "profiles", "mfma_shapes", "toeplitz.py"))
    tz = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tz)
    for h in range(1, 32, 2):
        for w in range(1, 32, 2):
            assert tz.window_useful(w, h) == pytest.approx(h * w / (32.0 * host.tsplit_windows(h, w)))
    # the row forms: w taps of a K-wide window per row, M outputs per block row
    assert tz.row_useful(15, 16, 32) == pytest.approx(15 / 32)
    assert tz.row_useful(19, 16, 32) == pytest.approx(19 / 64)
