"""RCCL (torch.distributed "nccl" on ROCm) on the GPU at world size 1
(VERDICT r3 #4): the reducer exchange of the multi-GPU path and bench.py's
N>1 code path run through RCCL itself, each in its own child process (one
rank on GPU 0), and must return exactly what the one-process path returns.
The 8-GPU scaling run itself belongs to the driver."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_world1_exchange():
    p = subprocess.run([sys.executable, os.path.join(REPO, "tests", "rccl_world1.py")], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    print(res)
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["detections"] > 0
    assert res["gather_counts_equal"] and res["gather_rows_bitexact"] and res["gather_on_device"] == "cuda"
    assert res["empty_ok"] and res["records_bitexact"]


@pytest.mark.gpu
def test_bench_dist_path_rccl_world1():
    """bench.py's N>1 step (detect + pack_rows + all_gather_detections over
    RCCL, barriers, max-over-ranks timing) launched by torch.distributed.run
    with one rank; the line names the exchange and one physical GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--dist", "--steps", "2", "--warmup", "1", "--batch", "4",
           "--no-cpu-baseline", "--no-xcorr-classes"]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=300, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 1 and out["physical_gpus"] == 1
    assert out["exchange"].startswith("nccl all-gather")
    assert out["value"] > 0
