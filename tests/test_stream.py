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


@pytest.mark.parametrize("world", [2, 3])
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
