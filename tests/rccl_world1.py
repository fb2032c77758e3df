"""Child process of tests/test_gpu_rccl.py: torch.distributed over RCCL
("nccl" on ROCm) at world size 1 on GPU 0 (TCP store on 127.0.0.1), driving
the reducer exchange of the N>1 path (driver.all_gather_detections,
mapreduce.gather_records) on real TMREngine.detect output, and comparing
each with the one-process result.  Prints one JSON line."""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
from tmr_import import load_package  # noqa: E402

tmr = load_package()
import oracle  # noqa: E402
from tmr_amd import driver, mapreduce, synth  # noqa: E402


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    P = oracle.reference_weights(0, cin=32, emb=32)
    P["objectness_head.head.0.bias"] = torch.tensor([0.5])
    eng = tmr.TMREngine({k: v.to(dev) for k, v in P.items()}, tmr.PathConfig(emb_dim=32))
    feats = torch.from_numpy(synth.sam_features(21, 5, 32, 16, 16)).to(dev)
    ex, _ = synth.exemplar_set(22, 5, 3, 32, 32, 3, 7)
    L, Bx, R = eng.detect(feats, ex, 0.5, 0.5)
    counts, rows = driver.pack_rows(L, Bx, R)
    g_counts, g_rows = driver.all_gather_detections(counts, rows)
    torch.cuda.synchronize()
    res["detections"] = int(rows.shape[0])
    res["gather_counts_equal"] = bool(torch.equal(g_counts.cpu(), counts.cpu()))
    res["gather_rows_bitexact"] = bool(np.array_equal(g_rows.cpu().numpy().view(np.uint32),
                                                      rows.cpu().numpy().view(np.uint32)))
    res["gather_on_device"] = g_rows.device.type
    # an image with no detections and a rank-local empty batch
    e_counts, e_rows = driver.all_gather_detections(torch.zeros(0, dtype=torch.int32, device=dev),
                                                    torch.zeros((0, driver.ROW), device=dev))
    res["empty_ok"] = e_counts.numel() == 0 and e_rows.shape[0] == 0
    # the streaming shuffle (per-tar records, fp64)
    rec = np.random.default_rng(3).normal(size=(9, mapreduce.REC))
    got = mapreduce.gather_records(rec)
    res["records_bitexact"] = bool(np.array_equal(got.view(np.uint64), rec.view(np.uint64)))
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
