"""Multi-process data-parallel driver on CPU (gloo, world_size 2, 3 and 8).

The per-rank compute here is the CPU oracle (tests may use it as the
checker); the product's GPU run uses TMREngine.detect with the same driver
code and the nccl (RCCL) backend.  Checks: sharding covers every image once,
the all-gather returns every rank's detections in global image order, and
the result equals a single-process run -- including 8 ranks (the node's GPU
count, rehearsed on CPU) over 13 images, where ranks hold 1 or 2 images and
(batch 1) the short ones run out and contribute empty batches to the later
rounds' all-gathers, and over 5 images, where 3 ranks hold none at all.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_REPO, os.path.join(_REPO, "oracle")):  # spawned workers skip conftest
    if _p not in sys.path:
        sys.path.insert(0, _p)
from tmr_import import load_package  # noqa: E402

load_package()
import oracle  # noqa: E402
from tmr_amd import driver, synth  # noqa: E402

CIN, EMB, HF = 16, 16, 8


def _detect_oracle(P):
    def fn(feats, ex):
        L, Bx, R = [], [], []
        for b in range(feats.shape[0]):
            ls, bs, rs = [], [], []
            for e in range(ex.shape[1]):
                exm = [torch.from_numpy(ex[b, e:e + 1])]
                o, bb, _, _ = oracle.forward_torch(feats[b:b + 1], exm, P)
                prob = oracle.sigmoid_cr(o[0][0, 0].numpy())
                l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [bb[0][0].numpy()], exm, 0.5)
                ls.append(l_[0]); bs.append(b_[0]); rs.append(r_[0])
            l2, b2, r2 = oracle.nms_lists([np.concatenate(ls)], [np.concatenate(bs)],
                                          [np.concatenate(rs)], 0.5)
            L.append(torch.from_numpy(l2[0])); Bx.append(torch.from_numpy(b2[0]))
            R.append(torch.from_numpy(r2[0]))
        return L, Bx, R
    return fn


def _setup(n=7):
    P = oracle.reference_weights(0, cin=CIN, emb=EMB)
    P["objectness_head.head.0.bias"] = torch.tensor([0.3])
    feats = torch.from_numpy(synth.sam_features(3, n, CIN, HF, HF))
    ex, _ = synth.exemplar_set(4, n, 2, 2 * HF, 2 * HF, 3, 5)
    return P, feats, ex, n


def _worker(rank, world, port, q, n=7, batch=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    P, feats, ex, n = _setup(n)
    counts, rows = driver.run_sharded(_detect_oracle(P), lambda s, e: (feats[s:e], ex[s:e]), n,
                                      batch=batch, rank=rank, world=world)
    q.put((rank, counts, [r.numpy() for r in rows]))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,n,batch", [(2, 7, 2), (3, 7, 2), (8, 13, 2), (8, 13, 1), (8, 5, 1)])
def test_sharded_driver_gloo(world, n, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, n, batch)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference run
    P, feats, ex, n = _setup(n)
    c1, r1 = driver.run_sharded(_detect_oracle(P), lambda s, e: (feats[s:e], ex[s:e]), n,
                                batch=batch, rank=0, world=1)
    assert (c1 >= 1).all()
    for rank, counts, rows in res:
        assert np.array_equal(counts, c1), rank
        for i in range(n):
            assert np.array_equal(rows[i], r1[i].numpy()), (rank, i)


def test_shard_range_covers_once():
    for n in (0, 1, 7, 64, 744):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, e = driver.shard_range(n, r, world)
                seen.extend(range(s, e))
                assert abs((e - s) - n / world) < 1
            assert seen == list(range(n))


def test_reducer_table_and_categories():
    assert driver.category_of("Easy_188.tar") == "Easy"
    assert driver.category_of("Hard_3.tar") == "Hard"
    assert driver.category_of("foo.tar") == "Unknown"
    t = driver.reducer_table(["Easy", "Hard", "Easy"], [3, 5, 1])
    lines = t.splitlines()
    assert lines[0].startswith("CATEGORY")
    assert "Easy" in lines[2] and "4" in lines[2]
