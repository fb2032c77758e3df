"""Assemble the correlation kernels' rocprofv3 sweep (profiles/gpu_xcorr_sweep.sh)
into profiles/xcorr_crossover.json and the engine's cost table
(tmr_amd/xcorr_cost.json).

Each regime (map size, images x exemplars, operand precision) was run as
`kbench_xcorr.py --reps R` under rocprofv3 once per counter pass (FETCH_SIZE,
WRITE_SIZE, the SQ/GRBM group) and once with --kernel-trace.  kbench launches
each (k, algo) 1 + R times in the order it prints its JSON lines, so the
correlation dispatches of a pass, in dispatch order, split into consecutive
groups of 1 + R; the first launch of a group (cold) is dropped.

Per (regime, algo, k): the kernel-trace duration (ms per launch), the HBM bytes
moved (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md), their rate against
the 8 TB/s peak, MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x the
per-XCD GPU cycles), VALU instructions and the effective clock.  The crossover
rule (engine.xcorr_choice) takes the per-k launch durations of this table; the
counters say which roof binds each point (hbm_frac near 0.8 of peak = HBM bound,
i.e. the ~6.3 TB/s achievable; rising VALU instructions and falling HBM rate =
compute bound).

    python profiles/xcorr_sweep_assemble.py <sweep-dir> <round-label>
"""
import csv
import glob
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PAT = re.compile(r"xcorr_(rows|mfma)_kernel")


def dispatches(d):
    """{dispatch id: (kernel name, start, end, {counter: value})} of the
    correlation kernels in one rocprofv3 output directory."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if not PAT.search(row["Kernel_Name"]):
                continue
            key = int(row["Dispatch_Id"])
            rec = out.setdefault(key, [row["Kernel_Name"], int(row["Start_Timestamp"]),
                                       int(row["End_Timestamp"]), {}])
            rec[3][row["Counter_Name"]] = rec[3].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if PAT.search(row["Kernel_Name"]):
                out.setdefault(int(row["Dispatch_Id"]), [row["Kernel_Name"], int(row["Start_Timestamp"]),
                                                         int(row["End_Timestamp"]), {}])
    return [out[k] for k in sorted(out)]


def groups(d, lines, reps):
    ds = dispatches(d)
    n = 1 + reps
    if len(ds) != n * len(lines):
        raise SystemExit(f"{d}: {len(ds)} correlation dispatches for {len(lines)} (k, algo) points x {n}")
    res = []
    for i, ln in enumerate(lines):
        g = ds[i * n + 1:(i + 1) * n]
        want = "rows" if ln["algo"] == "valu" else "mfma"
        if not all(want in x[0] for x in g):
            raise SystemExit(f"{d}: dispatch group {i} is not the {ln['algo']} kernel")
        res.append(g)
    return res


def _buildinfo():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "tmr_buildinfo", os.path.join(REPO, "template-matching-and-regression-mapreduce_amd", "buildinfo.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def regime(d, reps):
    lines = [json.loads(x) for x in open(os.path.join(d, "kbench.jsonl")) if x.startswith("{")]
    lines = [x for x in lines if "error" not in x]
    per = {x["algo"] + ":" + x["k"]: dict(x) for x in lines}
    gt = groups(os.path.join(d, "trace"), lines, reps)
    for ln, g in zip(lines, gt):
        per[ln["algo"] + ":" + ln["k"]]["trace_ms"] = mean([(x[2] - x[1]) * 1e-6 for x in g])
    for p in ("fetch", "write", "core"):
        pd = os.path.join(d, p)
        if not os.path.isdir(pd):
            continue
        for ln, g in zip(lines, groups(pd, lines, reps)):
            r = per[ln["algo"] + ":" + ln["k"]]
            cs = {}
            for x in g:
                for c, v in x[3].items():
                    cs.setdefault(c, []).append(v)
            for c, v in cs.items():
                r.setdefault("counters", {})[c] = mean(v)
    for r in per.values():
        c = r.get("counters", {})
        ms = r.get("trace_ms")
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            r["hbm_bytes"] = 2 * 1024 * c["FETCH_SIZE"] + 1024 * c["WRITE_SIZE"]
            if ms:
                r["hbm_gbps_counted"] = r["hbm_bytes"] / ms / 1e6
                r["hbm_frac_counted"] = r["hbm_gbps_counted"] / 8000.0
        if "GRBM_GUI_ACTIVE" in c and ms:
            r["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                r["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
    return per


def main(sweep, label, reps=3):
    out = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "round": label, "regimes": {}}
    for d in sorted(glob.glob(os.path.join(sweep, "*"))):
        if os.path.isdir(d) and os.path.exists(os.path.join(d, "kbench.jsonl")):
            out["regimes"][os.path.basename(d)] = regime(d, reps)
    # the sources the swept kernels were built from: a kernel edit without a
    # re-sweep turns tests/test_abi_host.py's digest check red
    digest = _buildinfo().source_digest("xcorr")
    out["source_digest"] = digest
    with open(os.path.join(HERE, "xcorr_crossover.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    # the engine's table: per regime and algo, ms per launch by k
    cost = {"source": f"profiles/xcorr_crossover.json (rocprofv3 kernel trace, round {label})",
            "source_digest": digest, "regimes": {}}
    for name, per in out["regimes"].items():
        t = {}
        for key, r in per.items():
            algo, k = key.split(":")
            t.setdefault(algo, {})[int(k)] = r.get("trace_ms")
            meta = {m: r[m] for m in ("images", "E", "H", "prec")}
        cost["regimes"][name] = dict(meta, ms={a: sorted(v.items()) for a, v in t.items()})
    with open(os.path.join(REPO, "template-matching-and-regression-mapreduce_amd", "xcorr_cost.json"), "w") as fh:
        json.dump(cost, fh, indent=1)
    for name, per in out["regimes"].items():
        print(name)
        for key in sorted(per, key=lambda s: (int(s.split(":")[1]), s)):
            r = per[key]
            print(f"  {key:10s} {r.get('trace_ms', 0):8.3f} ms  hbm {r.get('hbm_frac_counted', 0):.3f}  "
                  f"mfma {r.get('mfma_busy', 0):.3f}  clk {r.get('clock_ghz', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
