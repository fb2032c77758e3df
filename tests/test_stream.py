"""Streaming map/reduce (mapper.py:34-142, reducer.py:34-94).

CPU: the reducer restatement reproduces the reference reducer.py's stdout
and stderr byte for byte on the golden cases (tests/golden/reducer_cases.json,
made by oracle/make_golden_stream.py running the reference), the mapper line
protocol, the shard split, and the gloo world-2/3 map + shuffle equal a
single-process run.  GPU: tmr_feature_stats vs the mapper's numpy statistics
(oracle.mapper_stats) and the end-to-end map phase with detections.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_REPO, os.path.join(_REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
from tmr_import import load_package  # noqa: E402

load_package()
import oracle  # noqa: E402
from tmr_amd import mapreduce as mr, synth  # noqa: E402

GOLDEN = os.path.join(_REPO, "tests", "golden")


def _cases():
    with open(os.path.join(GOLDEN, "reducer_cases.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("case", ["sorted", "interleaved", "malformed", "zero_count", "progress", "empty"])
def test_reducer_matches_reference_bytes(case):
    c = _cases()[case]
    so, se = mr.reduce_lines(c["input"])
    assert so == c["stdout"]
    assert se == c["stderr"]


def test_mapper_line_protocol():
    stats = [oracle.mapper_stats(synth.sam_features(i, 1, 8, 4, 4)) for i in range(4)]
    sums, cnt = oracle.mapper_tar_sums(stats)
    assert mr.mapper_line("Easy", sums, cnt) == oracle.mapper_line("Easy", sums, cnt)
    assert mr.mapper_line("Hard", sums, cnt, 17).endswith(f",{cnt},17")
    # extended lines reduce with the extra columns; plain lines still parse
    so, _ = mr.reduce_lines(["Easy\t0.5,1.0,2.0,0.5,2,10", "Easy\t0.5,1.0,2.0,0.5,3,5"], detections=True)
    assert so.splitlines()[2].split("|")[-2:] == ["         15 ", "     3.00"]


def test_shard_split_and_categories():
    with open(os.path.join(GOLDEN, "list_tars.txt")) as fh:
        shards = [l.strip() for l in fh if l.strip()]
    assert len(shards) == 744
    counts = mr.shard_image_counts(shards)
    assert min(counts) >= 3 and max(counts) <= 6
    for world in (1, 2, 3, 8):
        rs = mr.weighted_ranges(counts, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(shards)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        tot = [sum(counts[s:e]) for s, e in rs]
        assert max(tot) - min(tot) <= 2 * max(counts)
    cats = {mr.category_of(s.replace(".tar", "")) for s in shards}
    assert cats == {"Easy", "Normal", "Hard"}
    assert mr.hadoop_sort(["b\t1", "a\t2", "b\t0", "a\t1"]) == ["a\t2", "a\t1", "b\t1", "b\t0"]


SHARDS = [f"{c}_{i}.tar" for c in ("Normal", "Easy", "Hard") for i in range(5)]


def _cpu_source(ids):
    f = np.concatenate([synth.sam_features(1000 + int(i), 1, 8, 6, 6) for i in ids])
    return torch.from_numpy(f), np.zeros((len(ids), 1, 4), np.float32)


def _cpu_stats(feats):
    return np.array([oracle.mapper_stats(f.numpy()) for f in feats])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    counts = mr.shard_image_counts(SHARDS, seed=3)
    rec = mr.run_mapper(SHARDS, counts, rank, world, _cpu_source, _cpu_stats, None, batch=4)
    q.put((rank, rec))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec = np.stack([np.arange(mr.REC, dtype=np.float64) + 100 * rank + 10 * j for j in range(rank % 3)]) \
        if rank % 3 else np.zeros((0, mr.REC))
    q.put((rank, mr.gather_records(rec)))
    dist.destroy_process_group()


def test_gather_records_uneven_world8_gloo():
    """The shuffle at the node's 8 ranks, holding 0, 1 or 2 records each
    (ranks with no shard contribute nothing): every rank receives all records
    in rank order (reducer.py:47-92 reads them in shard order)."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = np.stack([np.arange(mr.REC, dtype=np.float64) + 100 * r + 10 * j
                    for r in range(world) for j in range(r % 3)])
    for r in range(world):
        np.testing.assert_array_equal(got[r], ref)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_map_shuffle_gloo(world):
    counts = mr.shard_image_counts(SHARDS, seed=3)
    ref = mr.run_mapper(SHARDS, counts, 0, 1, _cpu_source, _cpu_stats, None, batch=4)
    # the single-process records equal the reference mapper's per-tar sums
    first = np.concatenate([[0], np.cumsum(counts)])
    for s in range(len(SHARDS)):
        ids = np.arange(first[s], first[s + 1])
        sums, cnt = oracle.mapper_tar_sums(_cpu_stats(_cpu_source(ids)[0]))
        assert list(ref[s, 1:5]) == sums and ref[s, 5] == cnt
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        np.testing.assert_array_equal(got[r], ref)
    lines = mr.hadoop_sort(mr.mapper_lines(SHARDS, got[0]))
    assert [l.split("\t")[0] for l in lines] == ["Easy"] * 5 + ["Hard"] * 5 + ["Normal"] * 5
    so, se = mr.reduce_lines(lines)
    assert so.count("\n") == 5 and "[ERROR]" not in se


# ---------------------------------------------------------------- GPU
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,H,W", [(5, 256, 64, 64), (3, 7, 5, 3), (1, 1, 1, 1), (0, 256, 64, 64)])
def test_feature_stats_vs_mapper_numpy(B, C, H, W):
    """mean/std: fp64-evaluated, rounded once to fp32 -- numpy's float32
    pairwise sums agree to a few fp32 ulps (tolerance 8 ulp of the value's
    scale); max and sparsity exact."""
    f = synth.sam_features(11, B, C, H, W) if B else np.zeros((0, C, H, W), np.float32)
    if B:
        f[:, :, 0, 0] = 0.0  # exact zeros count as sparse (<= 0)
    got = mr.feature_stats(torch.from_numpy(f).to(DEV))
    assert got.shape == (B, 4)
    for b in range(B):
        m, s, x, p = oracle.mapper_stats(f[b])
        scale = max(abs(s), float(np.abs(f[b]).max()))
        assert abs(got[b, 0] - m) <= 8 * np.spacing(np.float32(scale)), (got[b, 0], m)
        assert abs(got[b, 1] - s) <= 8 * np.spacing(np.float32(s)) + 1e-30, (got[b, 1], s)
        assert got[b, 2] == x and got[b, 3] == p


@pytest.mark.gpu
def test_map_phase_gpu_with_detections():
    """run_mapper on the GPU (stats kernel + TMREngine.detect, small emb) vs
    the CPU oracle's per-tar records: counts and detections exact, sums
    within the stats tolerance."""
    from tmr_amd import PathConfig, TMREngine

    shards = SHARDS[:6]
    counts = mr.shard_image_counts(shards, seed=5)
    P = oracle.reference_weights(0, cin=32, emb=32)
    P["objectness_head.head.0.bias"] = torch.tensor([0.5])
    eng = TMREngine({k: v.to(DEV) for k, v in P.items()}, PathConfig(emb_dim=32))

    def src(ids):
        f = np.concatenate([synth.sam_features(2000 + int(i), 1, 32, 8, 8) for i in ids])
        ex = np.concatenate([synth.exemplar_set(3000 + int(i), 1, 2, 16, 16, 3, 5)[0] for i in ids])
        return torch.from_numpy(f).to(DEV), ex

    rec = mr.run_mapper(shards, counts, 0, 1, src, mr.feature_stats,
                        lambda f, ex: eng.detect(f, ex, 0.5, 0.5), batch=5)
    first = np.concatenate([[0], np.cumsum(counts)])
    for s in range(len(shards)):
        ids = np.arange(first[s], first[s + 1])
        f, ex = src(ids)
        f = f.cpu()
        sums, cnt = oracle.mapper_tar_sums([oracle.mapper_stats(x.numpy()) for x in f])
        dets = 0
        for b in range(len(ids)):
            ls, bs, rs = [], [], []
            for e in range(ex.shape[1]):
                exm = [torch.from_numpy(ex[b, e:e + 1])]
                o, bb, _, _ = oracle.forward_torch(f[b:b + 1], exm, P)
                prob = oracle.sigmoid_cr(o[0][0, 0].numpy())
                l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [bb[0][0].numpy()], exm, 0.5)
                ls.append(l_[0]); bs.append(b_[0]); rs.append(r_[0])
            _, bo, _ = oracle.nms_lists([np.concatenate(ls)], [np.concatenate(bs)],
                                        [np.concatenate(rs)], 0.5)
            dets += bo[0].shape[0]
        assert rec[s, 5] == cnt and rec[s, 6] == dets
        np.testing.assert_allclose(rec[s, 1:5], sums, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------- feature cache (§8f f3)
def _feature_tree(root, shards, seed=40, C=8, h=6):
    """The reference mapper's output layout: <root>/<Category>/<tar stem>/<image>.npy [1,C,h,h]."""
    rng = np.random.default_rng(seed)
    for si, name in enumerate(shards):
        stem = name.replace(".tar", "")
        d = os.path.join(root, mr.category_of(stem), stem)
        os.makedirs(d, exist_ok=True)
        for j in range(int(rng.integers(0, 4))):  # 0..3 images (0: the tar emits no line)
            np.save(os.path.join(d, f"img_{j}.npy"),
                    synth.sam_features(100 * si + j, 1, C, h, h))


def test_npy_feature_source_map(tmp_path):
    shards = SHARDS[:7]
    _feature_tree(str(tmp_path), shards)
    src = mr.NpyFeatureSource(str(tmp_path), shards, torch.device("cpu"), 2, 3, 5, 0,
                              exemplars={"Normal_1/img_0": [[0.1, 0.1, 0.3, 0.3]]})
    assert len(src.counts) == len(shards) and sum(src.counts) == len(src.files)
    rec = mr.run_mapper(shards, src.counts, 0, 1, src, _cpu_stats, None, batch=2)
    for s, name in enumerate(shards):
        stem = name.replace(".tar", "")
        fs = sorted(os.listdir(os.path.join(str(tmp_path), mr.category_of(stem), stem)))
        stats = [oracle.mapper_stats(np.load(os.path.join(str(tmp_path), mr.category_of(stem), stem, f)))
                 for f in fs]
        sums, cnt = oracle.mapper_tar_sums(stats)
        assert rec[s, 5] == cnt and list(rec[s, 1:5]) == sums
    lines = mr.mapper_lines(shards, rec)
    assert len(lines) == sum(1 for c in src.counts if c > 0)  # empty tars emit nothing (mapper.py:127)
    i = src.keys.index("Normal_1/img_0")
    _, ex = src([i])
    np.testing.assert_array_equal(ex[0], np.float32([[0.1, 0.1, 0.3, 0.3]] * 2))


def test_load_weights_lightning_prefix(tmp_path):
    P = oracle.reference_weights(0, cin=8, emb=8)
    sd = {"model." + k: v for k, v in P.items()}
    sd["model.encoder.backbone.w"] = torch.zeros(2)
    torch.save({"state_dict": sd, "epoch": 3}, str(tmp_path / "c.ckpt"))
    got = mr.load_weights(str(tmp_path / "c.ckpt"), torch.device("cpu"))
    assert set(got) == set(P)
    for k in P:
        assert torch.equal(got[k], P[k].float())


@pytest.mark.gpu
def test_stream_cli_on_feature_tree(tmp_path, capsys):
    """stream.py main() on the mapper's feature tree with a checkpoint: the
    reducer table equals the CPU oracle's (statistics within the kernel's
    fp32-rounding tolerance at 4 decimals, counts exact)."""
    shards = SHARDS[:6]
    root = tmp_path / "feat"
    _feature_tree(str(root), shards, C=32, h=8)
    P = oracle.reference_weights(0, cin=32, emb=32)
    torch.save(P, str(tmp_path / "w.pt"))
    lst = tmp_path / "list.txt"
    lst.write_text("".join(s + "\n" for s in shards))
    mr.main(["--list", str(lst), "--features-root", str(root), "--ckpt", str(tmp_path / "w.pt"),
             "--exemplars", "2", "--kmax", "5", "--detections", "--mapper-out", str(tmp_path / "m.txt")])
    out = capsys.readouterr().out
    src = mr.NpyFeatureSource(str(root), shards, torch.device("cpu"), 2, 3, 5, 0)
    rec = mr.run_mapper(shards, src.counts, 0, 1, src, _cpu_stats, None, batch=64)
    lines = open(str(tmp_path / "m.txt")).read().splitlines()
    ref_lines = mr.hadoop_sort(mr.mapper_lines(shards, rec))
    assert [l.split("\t")[0] for l in lines] == [l.split("\t")[0] for l in ref_lines]
    for l, r in zip(lines, ref_lines):
        got = [float(v) for v in l.split("\t")[1].split(",")]
        exp = [float(v) for v in r.split("\t")[1].split(",")]
        assert got[4] == exp[4] and got[2] == exp[2] and got[3] == exp[3]  # count, max, sparsity exact
        np.testing.assert_allclose(got[:2], exp[:2], rtol=1e-6, atol=1e-6)
    assert out.splitlines()[0].startswith("CATEGORY")


# ---------------------------------------------------------------- backbone producer (§8f f3)
def _png_bytes(arr, mode):
    from PIL import Image
    buf = __import__("io").BytesIO()
    Image.fromarray(arr, mode).save(buf, format="PNG")
    return buf.getvalue()


def _jpeg_bytes(arr):
    from PIL import Image
    buf = __import__("io").BytesIO()
    Image.fromarray(arr, "RGB").save(buf, format="JPEG", quality=90)
    return buf.getvalue()


def _tar_tree(root, shards, seed=7):
    """Tar shards as the reference's Gen_Tar_Data ones: images at any depth,
    mixed formats/modes/case, plus a non-image and an undecodable .png."""
    import io
    import tarfile
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    n_ok = []
    for si, name in enumerate(shards):
        members = []
        k = int(rng.integers(0, 4))
        for j in range(k):
            h, w = int(rng.integers(20, 90)), int(rng.integers(20, 90))
            kind = (si + j) % 4
            if kind == 0:
                members.append((f"img_{j}.png", _png_bytes(rng.integers(0, 256, (h, w, 3), dtype=np.uint8), "RGB")))
            elif kind == 1:
                members.append((f"sub/dir/IMG_{j}.PNG", _png_bytes(rng.integers(0, 256, (h, w), dtype=np.uint8), "L")))
            elif kind == 2:
                members.append((f"a/img_{j}.jpeg", _jpeg_bytes(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))))
            else:
                members.append((f"img_{j}.Jpg", _png_bytes(rng.integers(0, 256, (h, w, 4), dtype=np.uint8), "RGBA")))
        members.append(("notes.txt", b"not an image"))
        if si % 3 == 0:
            members.append(("broken.png", b"\x89PNG garbage"))
        with tarfile.open(os.path.join(root, name), "w") as tf:
            for mname, data in members:
                ti = tarfile.TarInfo(mname)
                ti.size = len(data)
                tf.addfile(ti, io.BytesIO(data))
        n_ok.append(k)
    return n_ok


class _PoolBackbone(torch.nn.Module):
    """A small deterministic stand-in encoder: 16x16 average pooling + a fixed
    1x1 projection to C channels (the real SAM encoder is registered the same way)."""

    def __init__(self, C=8):
        super().__init__()
        g = torch.Generator().manual_seed(5)
        self.proj = torch.nn.Conv2d(3, C, 1)
        with torch.no_grad():
            self.proj.weight.copy_(torch.randn(C, 3, 1, 1, generator=g))
            self.proj.bias.copy_(torch.randn(C, generator=g) * 0.1)
        self.num_channels = C

    def forward(self, x):
        return self.proj(torch.nn.functional.avg_pool2d(x, 16))


def test_tar_images_and_preprocess(tmp_path):
    """mapper.py:22-32 + :85-88: image members at any depth, extension test
    case-insensitive, non-images ignored, undecodable images dropped; the
    preprocessing is PIL RGB -> resize (PIL's default filter, bicubic in the
    Pillow of this image and of the reference's pinned environment) -> /255
    -> [1,3,H,W] float32.  Parity unpinned beyond PIL itself (onnxruntime, which
    the reference mapper imports at module load, is absent here)."""
    from PIL import Image
    shards = ["Easy_0.tar", "Hard_1.tar", "Normal_2.tar", "Easy_3.tar"]
    n_ok = _tar_tree(str(tmp_path), shards)
    for si, name in enumerate(shards):
        names = [m for m, _ in mr.tar_images(str(tmp_path / name))]
        assert names == sorted(names)
        assert "notes.txt" not in names
        assert len(names) == n_ok[si] + (1 if si % 3 == 0 else 0)
    src = mr.TarImageSource(str(tmp_path), shards, _PoolBackbone(), torch.device("cpu"), 2, 3, 5, 0,
                            input_shape=(64, 48))
    assert src.counts == n_ok
    for i in range(len(src.items)):
        path, member, _, plain = src.items[i]
        assert plain
        x = src._read(i)
        assert x.shape == (1, 3, 48, 64) and x.dtype == np.float32
        import tarfile
        with tarfile.open(path) as tf:
            img = Image.open(tf.extractfile(member.name)).convert("RGB")
        ref = np.asarray(img.resize((64, 48), Image.Resampling.BICUBIC)).astype(np.float32) / np.float32(255.0)
        np.testing.assert_array_equal(x[0], ref.transpose(2, 0, 1))
    assert mr.preprocess_image(b"garbage") is None


def test_tar_reads_do_not_rescan_headers(tmp_path, monkeypatch):
    """an image read must not re-read the shard's headers (a
    lookup by name walks them all: O(n^2) per shard).  After listing, reading
    every image of a plain shard opens no TarFile; a gzip shard (no direct
    offsets) is read through one TarFile per thread, by TarInfo, with the
    same bytes."""
    import gzip
    import shutil
    import tarfile
    shards = ["Easy_0.tar", "Hard_1.tar"]
    _tar_tree(str(tmp_path), shards)
    src = mr.TarImageSource(str(tmp_path), shards, _PoolBackbone(), torch.device("cpu"), 2, 3, 5, 0,
                            input_shape=(32, 32))
    opened = []
    real_open = tarfile.open
    monkeypatch.setattr(tarfile, "open", lambda *a, **k: opened.append(a) or real_open(*a, **k))
    plain_bytes = [mr.read_member(p, m, pl) for p, m, _, pl in src.items]
    for i in range(len(src.items)):
        src._read(i)
    assert opened == []
    # the same shard gzip-compressed
    gz = tmp_path / "gz"
    gz.mkdir()
    with open(tmp_path / "Easy_0.tar", "rb") as fi, gzip.open(gz / "Easy_0.tar", "wb") as fo:
        shutil.copyfileobj(fi, fo)
    plain, members = mr.tar_members(str(gz / "Easy_0.tar"))
    assert not plain
    tls = mr.TarHandles()
    opened.clear()
    got = [mr.read_member(str(gz / "Easy_0.tar"), m, plain, tls) for m in members]
    assert len(opened) == 1 and len(tls) == 1
    want = [b for (p, _, _, _), b in zip(src.items, plain_bytes) if p.endswith("Easy_0.tar")]
    decodable = {m.name for p, m, _, _ in src.items if p.endswith("Easy_0.tar")}
    assert [g for g, m in zip(got, members) if m.name in decodable] == want
    # every handle is released by close(); the next read reopens
    handle = tls.get(str(gz / "Easy_0.tar"))
    tls.close()
    assert len(tls) == 0 and handle.closed
    assert mr.read_member(str(gz / "Easy_0.tar"), members[0], plain, tls) == got[0]
    tls.close()
    # a source over the gzip shard holds no handle after its scan, and close()
    # releases the readers' handles
    src2 = mr.TarImageSource(str(gz), ["Easy_0.tar"], _PoolBackbone(), torch.device("cpu"), 2, 3, 5, 0,
                             input_shape=(32, 32))
    assert len(src2._tls) == 0
    src2([0])
    assert len(src2._tls) >= 1
    src2.close()
    assert len(src2._tls) == 0


def test_tar_source_feature_cache_roundtrip(tmp_path):
    """The producer's features, written as the mapper's .npy cache, read back
    by NpyFeatureSource: same files/layout, bit-identical features and
    per-tar records (CPU stats)."""
    shards = [f"{c}_{i}.tar" for c in ("Normal", "Easy", "Hard") for i in range(3)]
    _tar_tree(str(tmp_path / "tars"), shards, seed=11)
    bb = _PoolBackbone().eval()
    src = mr.TarImageSource(str(tmp_path / "tars"), shards, bb, torch.device("cpu"), 2, 3, 5, 0,
                            write_root=str(tmp_path / "feat"), workers=2, input_shape=(128, 128))
    rec = mr.run_mapper(shards, src.counts, 0, 1, src, _cpu_stats, None, batch=3)
    src.close()
    back = mr.NpyFeatureSource(str(tmp_path / "feat"), shards, torch.device("cpu"), 2, 3, 5, 0)
    assert back.counts == src.counts
    assert sorted(back.keys) == sorted(src.keys)
    for i, key in enumerate(src.keys):
        j = back.keys.index(key)
        f_back, _ = back([j])
        with torch.no_grad():
            f_new = bb(torch.from_numpy(src._read(i)))
        assert f_back.shape == (1, 8, 8, 8)
        assert torch.equal(f_back, f_new)
    rec2 = mr.run_mapper(shards, back.counts, 0, 1, back, _cpu_stats, None, batch=3)
    # same per-tar sums up to the image order inside a tar (sorted member
    # paths vs sorted file stems)
    np.testing.assert_allclose(rec2, rec, rtol=1e-12, atol=0)


@pytest.mark.gpu
def test_stream_cli_tar_producer(tmp_path, capsys):
    """stream.py main() over tar shards through a registered backbone on the
    GPU, writing the feature cache; a second run over that cache gives the
    same mapper lines (the stats kernel on identical features)."""
    from tmr_amd import register_backbone, unregister_backbone
    shards = [f"{c}_{i}.tar" for c in ("Normal", "Easy", "Hard") for i in range(3)]
    _tar_tree(str(tmp_path / "tars"), shards, seed=13)
    register_backbone("test_pool", lambda args: _PoolBackbone(C=32))
    try:
        lst = tmp_path / "list.txt"
        lst.write_text("".join(s + "\n" for s in shards))
        common = ["--list", str(lst), "--exemplars", "2", "--kmax", "5", "--stats-only"]
        mr.main(common + ["--tars-root", str(tmp_path / "tars"), "--backbone", "test_pool",
                          "--write-features", str(tmp_path / "feat"), "--mapper-out", str(tmp_path / "a.txt")])
        out_a = capsys.readouterr().out
        mr.main(common + ["--features-root", str(tmp_path / "feat"), "--mapper-out", str(tmp_path / "b.txt")])
        out_b = capsys.readouterr().out
    finally:
        unregister_backbone("test_pool")
    a = open(str(tmp_path / "a.txt")).read().splitlines()
    b = open(str(tmp_path / "b.txt")).read().splitlines()
    assert len(a) == len(b) > 0
    for la, lb in zip(a, b):
        assert la.split("\t")[0] == lb.split("\t")[0]
        va = [float(v) for v in la.split("\t")[1].split(",")]
        vb = [float(v) for v in lb.split("\t")[1].split(",")]
        assert va[4] == vb[4]
        np.testing.assert_allclose(va, vb, rtol=1e-12)
    assert out_a.splitlines()[0].startswith("CATEGORY") and out_a == out_b


def test_sam_preprocessing():
    """extract_feature.py:49-66: longest side to the target (int(x * s + 0.5)),
    PIL bilinear, fp32 (x - mean) / std, zero pad right/bottom."""
    from PIL import Image
    rng = np.random.default_rng(3)
    arr = rng.integers(0, 256, (30, 50, 3), dtype=np.uint8)
    data = _png_bytes(arr, "RGB")
    x = mr.preprocess_image_sam(data, 64)
    assert x.shape == (1, 3, 64, 64) and x.dtype == np.float32
    newh, neww = int(30 * (64 / 50) + 0.5), int(50 * (64 / 50) + 0.5)
    assert (newh, neww) == (38, 64)
    r = np.asarray(Image.fromarray(arr).resize((neww, newh), Image.Resampling.BILINEAR)).astype(np.float32)
    mean = np.float32([123.675, 116.28, 103.53])
    std = np.float32([58.395, 57.12, 57.375])
    ref = (r - mean) / std
    np.testing.assert_array_equal(x[0, :, :newh, :neww], ref.transpose(2, 0, 1))
    assert not x[0, :, newh:, :].any()
    assert mr.preprocess_image_sam(b"garbage") is None
