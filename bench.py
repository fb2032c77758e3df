"""bench.py -- images/sec of the TMR match+regress+NMS hot path on MI355X.

Workload (BASELINE.json configs[1], "config B"): per GPU a batch of 64
synthetic SAM feature maps [64,256,64,64] fp32 (upsampled in-path to
128x128), 3 exemplars per image with templates 3x3..15x15, reference-init
weights (emb 512, fusion, 1-layer 3x3 decoders), cls 0.1 / IoU 0.5
(scripts/train/TMR_FSCD147.sh:20-21).  One step = the whole path for the
batch: upsample+proj, RoIAlign, xcorr, fused decoders+heads, peaks+decode,
NMS over each image's exemplar union (+ for N>1 the RCCL all-gather of
per-image counts and kept boxes that replaces the Hadoop reducer).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

`python bench.py --gpus N` (N > 1) outside a torch.distributed launch starts
the N rank processes itself (torch.distributed.run, 127.0.0.1, one per GPU)
before anything touches the GPU, and exits with their status; launched by
torchrun, WORLD_SIZE must equal --gpus.  The reference's counterparts are
Lightning DDP over all devices (main.py:108-119) and Hadoop's map-side
parallelism (mapper.py:51).

Prints one JSON line (rank 0).  `roofline` is the fused decoder kernel
(tmr_conv_heads, >98% of the path's FLOPs) timed with HIP events on its
launch stream; `cpu_baseline` is the CPU oracle (torch-CPU restatement of the
reference forward + C peaks/NMS) on a bounded sample, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))


def launch_plan(argv, env):
    """What `bench.py argv` must do about ranks, decided before torch or the
    package is imported: None = run here as this rank; a command list = start
    the N rank processes with it and exit with their status.  Raises
    SystemExit(2) when a torch.distributed launch disagrees with --gpus."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args(argv)[0].gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != n:
            print(f"bench.py: refusing to run: WORLD_SIZE={world} but --gpus {n}", file=sys.stderr)
            raise SystemExit(2)
        return None
    if n == 1:
        return None
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:  # a free rendezvous port
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


if __name__ == "__main__":
    _cmd = launch_plan(sys.argv[1:], os.environ)
    if _cmd is not None:  # this process never touches the GPU: the ranks are children
        sys.exit(subprocess.call(_cmd))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

tmr = load_package()
from tmr_amd import driver, synth  # noqa: E402

METRIC = "images/sec (whole node) match+regress+NMS; % HBM/MFMA roofline at 1/2/4/8 GPU"
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), spec
# dense fp16/bf16 MFMA: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (MI355X_MICROARCH.md, ~2.5 PF)
F16_PEAK_TFLOPS = 2516.6
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
# 16-bit MFMA terms per product of the split decoder kernel (conv_split.hip)
SPLIT_TERMS = {"fp32": 3, "bf16": 1, "f16": 1}
EMB, CIN, KS = 512, 256, 3

# BASELINE.json configs; B is the metric's headline workload
CONFIGS = {
    "B": dict(desc="config B: 64x SAM feats 256x64x64 (->128x128), 3 exemplars, templates 3x3-15x15, "
                   "fp32, cls 0.1, IoU 0.5", batch=64, E=3, hf=64, kmin=3, kmax=15, cls=0.1, iou=0.5),
    "A": dict(desc="config A (demo.py shape): 1 image, SAM feats 256x64x64, 3 exemplars (k 7/11/15), "
                   "fp32, cls 0.7, IoU 0.5", batch=1, E=3, hf=64, kmin=7, kmax=15, cls=0.7, iou=0.5),
    "D": dict(desc="config D (RPINE streaming shape): 64x SAM feats 256x64x64, 1 exemplar, "
                   "templates 3x3-15x15, fp32, cls 0.4, IoU 0.5", batch=64, E=1, hf=64, kmin=3,
              kmax=15, cls=0.4, iou=0.5),
    "E": dict(desc="config E (large-pattern stress): 8x SAM feats 256x96x96 (->192x192), 16 exemplars, "
                   "templates 3x3-31x31, fp32, cls 0.1, IoU 0.5", batch=8, E=16, hf=96, kmin=3, kmax=31,
              cls=0.1, iou=0.5),
    "C": dict(desc="config C (FSCD-147 eval shape): 64x SAM feats 256x64x64 (->128x128), 3 shots, "
                   "templates 3x3-15x15, bf16 MFMA decoders (fp32 accumulate), cls 0.25, IoU 0.5",
              batch=64, E=3, hf=64, kmin=3, kmax=15, cls=0.25, iou=0.5, precision="bf16"),
}
H = W = 128  # set from the config in main()


def decoder_flops_per_unit() -> float:
    """Algorithmic FLOPs of the two 3x3 1024->1024 decoders per (image,
    exemplar) unit: 2 * H*W * N(=2048) * K(=1024*9)."""
    return 2.0 * H * W * (2 * 2 * EMB) * (2 * EMB * KS * KS)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """The cores this process may run on: its CPU affinity, capped by a
    cgroup-v2 CPU quota (a GPU box's share of a larger host: os.cpu_count()
    counts the whole machine there, and more threads than the quota would
    only time-slice)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(P, feats, ex, seconds: float, cls: float, iou: float):
    """The reference forward on the host cores: torch-CPU restatement
    (oracle/oracle.py, op for op the reference's ATen calls, one full forward
    per exemplar like demo.py:111) + C peaks/NMS.  Bounded by `seconds`.
    Threads: every core available to the process."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    threads = host_cores()
    torch.set_num_threads(threads)
    Pc = {k: v.detach().cpu() for k, v in P.items()}
    t0 = time.perf_counter()
    n = 0
    while n < feats.shape[0]:
        f = torch.from_numpy(feats[n:n + 1])
        Ls, Bs, Rs = [], [], []
        for e in range(ex.shape[1]):
            exm = [torch.from_numpy(ex[n, e:e + 1])]
            with torch.no_grad():
                o, b, _, _ = oracle.forward_torch(f, exm, Pc)
            prob = o[0][0, 0].sigmoid().numpy()
            l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [b[0][0].numpy()], exm, cls)
            Ls.append(l_[0]); Bs.append(b_[0]); Rs.append(r_[0])
        oracle.nms_lists([np.concatenate(Ls)], [np.concatenate(Bs)], [np.concatenate(Rs)], iou)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{n} image(s) x {ex.shape[1]} exemplars of the same workload, "
                      f"{dt:.1f} s, torch {torch.__version__} CPU ({threads} threads = the cores "
                      f"available to the process; the host reports {os.cpu_count()} CPUs, "
                      f"{cpu_model()})"}


def xcorr_by_class(eng, feats_d, ex, reps: int = 3):
    """The correlation kernel per template class (k <= 9: HBM-bound, k >= 11:
    VALU/MFMA-bound), each class's units of the batch in one
    tmr_xcorr launch, timed with HIP events on the launch stream (outside
    the timed region)."""
    from tmr_amd import host as _host
    B, E = ex.shape[:2]
    boxes = ex.reshape(-1, 4)
    ui = np.repeat(np.arange(B), E)
    fp, _ = eng.project(feats_d)
    Hm, Wm = fp.shape[-2:]
    ks = np.array([max(_host.template_size(b, Hm, Wm)[1:]) for b in boxes])
    out = {}
    for name, sel in (("k<=9", ks <= 9), ("k>=11", ks >= 11)):
        if not sel.any():
            continue
        eng.xcorr_events, eng.xcorr_split_events = [], []
        for _ in range(reps):
            eng.match(fp, ui[sel], boxes[sel])
        torch.cuda.synchronize()
        xs = float(np.mean([s_.elapsed_time(e_) for s_, e_ in eng.xcorr_events])) / 1e3
        eng.xcorr_events = None
        out[name] = {"units": int(sel.sum()), "algo": eng.last_xcorr_algo, "avg_launch_ms": round(1e3 * xs, 3),
                     "hbm_achieved": round(eng.last_xcorr_bytes / xs / 1e9, 1),
                     "hbm_frac": round(eng.last_xcorr_bytes / xs / 1e9 / HBM_PEAK_GBS, 4),
                     "valu_achieved": round(eng.last_xcorr_flops / xs / 1e12, 2),
                     "valu_frac": round(eng.last_xcorr_flops / xs / 1e12 / FP32_PEAK_TFLOPS, 4)}
        if eng.last_xcorr_algo == "mfma":  # the unit it runs on: dense 16-bit MFMA
            out[name]["mfma_frac"] = round(eng.last_xcorr_flops / xs / 1e12 / F16_PEAK_TFLOPS, 4)
    return out


PMC_FILE = os.path.join(REPO, "profiles", "pmc_by_config.json")
PEAKS_FILE = os.path.join(REPO, "profiles", "peaks_measured.json")


def measured_peaks():
    """The box's own peaks (profiles/peakbench), or None."""
    if not os.path.exists(PEAKS_FILE):
        return None
    with open(PEAKS_FILE) as fh:
        return json.load(fh)


def load_pmc(config: str, role: str):
    """The committed rocprofv3 PMC record (profiles/pmc_by_config.json,
    assembled by profiles/pmc_assemble.py) of this config's `role` kernel
    launch ("heads", "store", "xcorr") as (record, None), or (None, reason)
    when none was collected or it was collected on other kernel sources than
    this tree's (tmr_amd/buildinfo.py digest)."""
    from tmr_amd import buildinfo
    if not os.path.exists(PMC_FILE):
        return None, "no PMC file"
    with open(PMC_FILE) as fh:
        d = json.load(fh)
    rec = d.get("configs", {}).get(config, {}).get(role)
    if not isinstance(rec, dict):
        return None, "no PMC record for this config"
    have, want = rec.get("source_digest"), buildinfo.source_digest(role)
    if have != want:
        return None, (f"PMC record of round {d.get('round')} was collected on other kernel sources "
                      f"(digest {have} != this tree's {want}); re-run profiles/gpu_pmc.sh")
    return dict(rec, source=f"profiles/pmc_by_config.json round {d.get('round')}"), None


def physical_gpus(world: int, dev) -> int:
    """Distinct (host, device) pairs the ranks ran on: a rehearsal of N ranks
    on one card reports 1 here beside n_gpus = N."""
    if world == 1:
        return 1
    me = (socket.gethostname(), torch.cuda.get_device_properties(dev).name, dev.index,
          os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES", "")))
    allv = [None] * world
    dist.all_gather_object(allv, me)
    return len(set(allv))


def guard_fracs(obj, path="", hits=None):
    """Null every numeric *frac* field above 1 (a fraction above 1 means the
    figure it is taken against is not a ceiling) and list them."""
    hits = [] if hits is None else hits
    if isinstance(obj, dict):
        for k, v in obj.items():
            if "frac" in k and isinstance(v, (int, float)) and not isinstance(v, bool) and v > 1.0:
                hits.append(f"{path}{k}={v}")
                obj[k] = None
            else:
                guard_fracs(v, f"{path}{k}.", hits)
    return hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="B", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="images per GPU per step")
    ap.add_argument("--exemplars", type=int, default=None)
    ap.add_argument("--precision", default=None, choices=sorted(SPLIT_TERMS),
                    help="decoder arithmetic (default: the config's; fp32 = 3-term fp16 split)")
    ap.add_argument("--path", default="detect", choices=["detect", "module"],
                    help="detect: TMREngine.detect over the batch (B x E units per launch); module: "
                         "the reference's per-exemplar module calls (demo.py:106-130)")
    ap.add_argument("--no-graphs", action="store_true",
                    help="detect path: never replay the forward as a HIP graph (TMREngine.use_graphs)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed and run the reducer exchange even at one rank "
                         "(RCCL at world 1 on a 1-GPU box exercises the N>1 code path)")
    ap.add_argument("--no-xcorr-classes", action="store_true",
                    help="skip the per-template-class correlation launches after the timed region "
                         "(PMC passes: one launch per kernel role)")
    a = ap.parse_args()
    # the committed PMC records describe each config's own workload only
    own_options = (a.batch is None and a.exemplars is None and a.precision is None
                   and a.path == "detect")

    rank, world, local = driver.dist_env()
    # one process per GPU; a rehearsal with more ranks than GPUs (gloo on a
    # 1-GPU box) wraps the local rank onto the visible devices
    local = local % max(1, torch.cuda.device_count())
    backend = os.environ.get("TMR_BENCH_BACKEND", "nccl")  # "nccl" is RCCL on ROCm
    use_dist = world > 1 or a.dist
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    global H, W
    cfg = CONFIGS[a.config]
    H = W = 2 * cfg["hf"]
    P = synth.reference_state_dict(0, device=dev)
    prec = a.precision or cfg.get("precision", "fp32")
    eng = tmr.TMREngine(P, tmr.PathConfig(precision=prec))
    # A/B knob: TMR_BENCH_OUT_BF16=0 keeps the bf16 contract's f_TM plane in fp32
    eng.out_bf16 = os.environ.get("TMR_BENCH_OUT_BF16", "1") != "0"
    B = a.batch or cfg["batch"]
    E = a.exemplars or cfg["E"]
    feats = synth.sam_features(1000 + rank, B, CIN, H // 2, W // 2)
    ex, _ = synth.exemplar_set(2000 + rank, B, E, H, W, cfg["kmin"], cfg["kmax"])
    feats_d = torch.from_numpy(feats).to(dev)

    if a.path == "module":
        # the reference's module-level call sequence, line for line
        # (demo.py:106-130): one matching_net forward per exemplar (with its
        # relu(f_TM) and f[0] outputs), Get_pred_boxes, concat, one NMS
        from types import SimpleNamespace
        margs = SimpleNamespace(emb_dim=EMB, fusion=True, ablation_no_box_regression=False,
                                encoder="original", feature_upsample=True, no_matcher=False,
                                template_type="roi_align", squeeze=False, decoder_num_layer=1,
                                decoder_kernel_size=KS, modeltype="matching_net", backbone="features",
                                num_channels=CIN, precision=prec)
        model = tmr.build_model(margs)
        model.load_state_dict(P, strict=True)
        model = model.to(dev).eval()
        dummy = {"regression_ablation_b": False, "regression_ablation_c": False}

        def step():
            out = []
            with torch.no_grad():
                for b in range(B):
                    image = feats_d[b:b + 1]
                    # the image's exemplar boxes arrive with it, as from the
                    # reference's loader (fresh device tensors every image,
                    # DataLoader(pin_memory=True) + non_blocking copy)
                    ex_d = torch.from_numpy(ex[b]).pin_memory().to(dev, non_blocking=True)
                    pl, pb, pr = [], [], []
                    for exemplar in [[ex_d[e].unsqueeze(0)] for e in range(E)]:  # demo.py:106
                        po, preg, _, _ = model(image, exemplar)
                        _l, _b, _r = tmr.Get_pred_boxes(po, preg, exemplar, dummy, cfg["cls"], True)
                        pl.append(_l[0]); pb.append(_b[0]); pr.append(_r[0])
                    L_, _, _ = tmr.NMS([torch.concat(pl)], [torch.concat(pb)], [torch.concat(pr)],
                                       cfg["iou"])
                    out.append(L_[0])
            return out
    else:
        def step():
            L, Bx, R = eng.detect(feats_d, ex, cls_ths=cfg["cls"], iou_threshold=cfg["iou"])
            if use_dist:
                counts, rows = driver.pack_rows(L, Bx, R)
                driver.all_gather_detections(counts, rows)
            return L

    # detect path at small batches and the module path: the forward is
    # replayed as a HIP graph once its signature recurs (TMREngine.use_graphs); a replay records no
    # per-kernel events, so the kernels' HIP-event times then come from one
    # eager step after the timed loop (same kernels, same stream)
    eng.use_graphs = not a.no_graphs
    if a.path == "module":  # the module's engine replays each exemplar's forward
        model.engine().use_graphs = not a.no_graphs
    graphs = eng.use_graphs and (a.path == "module" or B * E <= eng.GRAPH_MAX_UNITS)
    for _ in range(a.warmup):
        step()
    if a.path == "module":
        eng = model.engine()  # the module's engine: its launches are the timed ones
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    if not graphs:
        eng.decoder_events = []
        eng.xcorr_events = []
        eng.xcorr_split_events = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        last = step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    graph_mode = eng.last_graph if graphs else None
    if graphs:  # the kernels' event times: one eager step after the timed loop
        eng.decoder_events, eng.xcorr_events, eng.xcorr_split_events = [], [], []
        step()
        torch.cuda.synchronize()
    dec_ms = [s.elapsed_time(e) for s, e in eng.decoder_events]
    xc_ms = [s.elapsed_time(e) for s, e in eng.xcorr_events]
    xs_ms = [s.elapsed_time(e) for s, e in eng.xcorr_split_events]
    eng.decoder_events = eng.xcorr_events = None
    kept = [int(x.shape[0]) for x in last]
    phys = physical_gpus(world, dev) if use_dist else 1

    if rank == 0:
        ms_step = 1e3 * elapsed / a.steps
        value = world * B / (elapsed / a.steps)
        flops = eng.last_decoder_flops  # executed FLOPs of the timed launch
        avg_s = float(np.mean(dec_ms)) / 1e3
        achieved = flops / avg_s / 1e12
        algo = eng.last_decoder_algo
        terms = SPLIT_TERMS[prec]
        peak = F16_PEAK_TFLOPS
        kernel_name = ("tmr_split_conv heads (direct implicit-GEMM decoder_b+decoder_o f_TM half "
                       "+ LeakyReLU + 1x1 heads, v_mfma_f32_16x16x32_%s)"
                       % ("bf16" if prec == "bf16" else "f16"))
        flops_basis = ("executed 16-bit MFMA work: %d term(s) x 2*H*W*N(2048)*K(512*9) per unit "
                       "(%s; the fp half runs once per image in a tmr_split_conv store launch and is "
                       "shared by its exemplars; unshared (E=1): K=(256+512)*9, the fp half folded through input_proj)"
                       % (terms, "fp32-grade 3-term fp16 split: hi*hi + lo*hi + hi*lo"
                          if terms == 3 else "one %s term" % prec))
        executed_achieved = achieved * terms
        # SURVEY.md 8d algorithmic FLOPs of the timed launch: the decoder
        # convs' f_TM half, 2*H*W*2048*(512*9) per unit (both halves when the
        # fp half is not shared, E = 1), independent of how the kernel
        # executes them (3-term split, folded projection, ...)
        units_per_launch = B * E if a.path == "detect" else 1
        alg_flops = 2.0 * H * W * (4 * EMB) * (EMB * KS * KS) * units_per_launch
        if eng.last_shared_flops == 0.0:
            alg_flops *= 2
        alg_achieved = alg_flops / avg_s / 1e12
        # whole path, EXECUTED MFMA-class work per step (SURVEY.md §7.3.2 / §8d:
        # when the fp half is shared across an image's exemplars, the fraction
        # is taken against the work actually executed): the decoders' f_TM
        # half per unit, their fp half (folded through input_proj, K = 256*9)
        # once per image when shared (else per unit), and the 1x1 projection
        # at the SAM features' size once per image; counted at one term
        shared = (eng.last_shared_flops > 0.0) if a.path == "detect" else E > 1
        S = H * W
        dec_tm = 2.0 * S * (4 * EMB) * (EMB * KS * KS) * B * E
        dec_fp = 2.0 * S * (4 * EMB) * (CIN * KS * KS) * (B if shared else B * E)
        proj = 2.0 * CIN * EMB * (S // 4) * B
        path_exec = dec_tm + dec_fp + proj
        path_ref = decoder_flops_per_unit() * B * E  # the reference's count: both halves per unit
        xc_flops, xc_bytes, xc_dram = eng.last_xcorr_flops, eng.last_xcorr_bytes, eng.last_xcorr_dram_bytes
        why_opts = "the run changes the config's options (--batch, --precision, ...)"
        pmc_heads, why_heads = load_pmc(a.config, "heads") if own_options else (None, why_opts)
        pmc_xc, why_xc = load_pmc(a.config, "xcorr") if own_options else (None, why_opts)
        if pmc_xc and pmc_xc.get("kernel_names") and not any(
                ("rows" if eng.last_xcorr_algo == "valu" else "mfma") in n for n in pmc_xc["kernel_names"]):
            pmc_xc, why_xc = None, "the PMC run measured the other correlation kernel"
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "images/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if prec == "bf16" else ("fp16" if prec == "f16" else "fp32"),
            "data": "synthetic (portable-PRNG SAM-like features, reference-init weights)",
            "config": {"workload": cfg["desc"], "config": a.config,
                       "images_per_gpu": B, "exemplars": E, "feature": [CIN, H // 2, W // 2],
                       "matching_map": [EMB, H, W], "parallelism": f"dp{world}",
                       "mean_kept_per_image": round(float(np.mean(kept)), 1),
                       "decoder": algo, "decoder_precision": prec, "path": a.path,
                       "hip_graph": graph_mode},
            "roofline": {"bound": "mfma", "kernel": kernel_name,
                         "achieved": round(alg_achieved, 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(alg_achieved / peak, 4),
                         "traffic": pmc_heads.get("hbm_bytes_per_launch") if pmc_heads else None,
                         "traffic_source": (pmc_heads["source"] + " (FETCH_SIZE x2 + WRITE_SIZE of this "
                                            "config's heads launch; its kernel-trace average %.3f ms)"
                                            % (1e3 * pmc_heads.get("avg_launch_s", float("nan"))))
                         if pmc_heads else f"null: {why_heads}",
                         "mfma_busy_pmc": round(pmc_heads["mfma_busy_frac"], 4)
                         if pmc_heads and "mfma_busy_frac" in pmc_heads else None,
                         "avg_launch_ms": round(1e3 * avg_s, 3),
                         "avg_launch_source": ("HIP events around the launch in the timed steps" if not graphs else
                                               "HIP events in one eager step after the timed loop (the timed "
                                               "steps replay a HIP graph, which records no per-kernel events)"),
                         "flops_per_launch": alg_flops,
                         "flops_basis": "algorithmic (SURVEY.md 8d): 2*H*W*N(2048)*K(512*9) per unit, the "
                                        "decoder_b+decoder_o conv over the f_TM half (x2 when E=1: both "
                                        "halves in this launch); peak = dense 16-bit MFMA",
                         "executed_achieved": round(executed_achieved, 2),
                         "executed_frac": round(executed_achieved / peak, 4),
                         "executed_basis": flops_basis,
                         "path_executed_tflop_per_step": round(path_exec / 1e12, 3),
                         "path_achieved": round(path_exec / (ms_step / 1e3) / 1e12, 2),
                         "path_frac": round(path_exec / (ms_step / 1e3) / 1e12 / peak, 4),
                         "path_basis": ("executed work per step at one term per product: decoders' f_TM "
                                        "half per unit + fp half (folded, K=256*9) %s + 1x1 projection "
                                        "per image, / step time / dense 16-bit MFMA peak"
                                        % ("once per image (shared by its exemplars)" if shared
                                           else "per unit")),
                         "path_reference_tflop_per_step": round(path_ref / 1e12, 2),
                         "path_reference_equiv_frac": round(path_ref / (ms_step / 1e3) / 1e12 / peak, 4)},
        }
        # the correlation kernel (SURVEY.md 8d "kernel 2"): HBM-bound for small
        # templates, VALU-bound for k >= 11; both fractions, algorithmic work
        xs = float(np.mean(xc_ms)) / 1e3
        xk = eng.last_xcorr_algo
        out["roofline_xcorr"] = {
            "kernel": ("tmr_xcorr MFMA (xcorr_mfma_kernel: 2-D window Toeplitz implicit GEMM on "
                       + ("v_mfma_f32_16x16x32_f16, 3-term fp16 split)" if prec == "fp32" else
                          "v_mfma_f32_16x16x32_%s, one %s term)" % (("bf16", "bf16") if prec == "bf16"
                                                                     else ("f16", "scaled fp16")))
                       if xk == "mfma" else
                       "tmr_xcorr VALU (xcorr_rows_kernel: LDS-blocked v_pk_fma_f32)")
                      + " + /hw + pad + scale + max|f_TM|; kernel chosen by the measured per-k cost model "
                        "(engine.XCORR_COST)",
            "algo": xk,
            "bound": "hbm" if cfg["kmax"] <= 9 else "valu",
            "avg_launch_ms": round(1e3 * xs, 3),
            "template_split_ms": round(float(np.mean(xs_ms)), 3) if xs_ms else None,
            "timing": "HIP events around the correlation kernel's launch alone on the engine stream; its "
                      "A-fragment pass (tmr_template_split, MFMA kernel only) is timed separately "
                      "(template_split_ms) and not in avg_launch_ms",
            "hbm_achieved": round(xc_bytes / xs / 1e9, 1), "hbm_peak": HBM_PEAK_GBS,
            "hbm_unit": "GB/s", "hbm_frac": round(xc_bytes / xs / 1e9 / HBM_PEAK_GBS, 4),
            "dram_min_bytes_per_launch": xc_dram,
            "dram_min_achieved": round(xc_dram / xs / 1e9, 1),
            "dram_min_frac": round(xc_dram / xs / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": pmc_xc.get("hbm_bytes_per_launch") if pmc_xc else None,
            "traffic_source": pmc_xc["source"] if pmc_xc else f"null: {why_xc}",
            "valu_achieved": round(xc_flops / xs / 1e12, 2), "valu_peak": FP32_PEAK_TFLOPS,
            "valu_unit": "TFLOP/s", "valu_frac": round(xc_flops / xs / 1e12 / FP32_PEAK_TFLOPS, 4),
            "basis": "hbm_*: SURVEY.md 8d bytes, read + write C*H*W fp32 per unit (the fp plane counted "
                     "once per unit); dram_min_*: the bytes the launch must move (each image's fp plane "
                     "read once for all its units, one f_TM plane written per unit); "
                     "2*C*(H-h+1)(W-w+1)*h*w FLOPs (SURVEY.md 8d)"}
        if not a.no_xcorr_classes:
            out["roofline_xcorr"]["by_class"] = xcorr_by_class(eng, feats_d, ex)
        mp = measured_peaks()
        if mp:  # the box's bare-loop figures: informational, not ceilings (see note)
            mk = "mfma_bf16_tflops" if prec == "bf16" else "mfma_f16_tflops"
            out["bare_loop"] = {
                "mfma_tflops": mp.get(mk),
                "mfma_implied_clock_ghz": round(2.4 * mp[mk] / F16_PEAK_TFLOPS, 3) if mp.get(mk) else None,
                "hbm_read_gbs": mp.get("hbm_read_gbs"), "hbm_copy_gbs": mp.get("hbm_copy_gbs"),
                "source": mp.get("source", "profiles/peaks_measured.json"),
                "note": ("profiles/peakbench: a bare MFMA loop holds a power-limited clock (implied above, "
                         "vs 2.4 GHz peak) that the decoder kernel exceeds (PMC ~1.9 GHz), so no MFMA "
                         "fraction is taken against it; fractions use the datasheet peaks")}
            if mp.get("hbm_copy_gbs"):
                out["roofline_xcorr"]["dram_min_frac_of_bare_loop_copy"] = \
                    round(xc_dram / xs / 1e9 / mp["hbm_copy_gbs"], 4)
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(P, feats, ex, a.cpu_seconds, cfg["cls"], cfg["iou"])
        else:
            out["cpu_baseline"] = None
        out["physical_gpus"] = phys
        out["exchange"] = (f"{dist.get_backend()} all-gather of counts + kept rows per step"
                           if use_dist else "none (one process)")
        hits = guard_fracs(out)
        if hits:
            out["frac_guard"] = "nulled (above 1): " + ", ".join(hits)
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
