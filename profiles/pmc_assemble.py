"""Assemble profiles/pmc_by_config.json from one measurement round's rocprofv3
--pmc passes (profiles/gpu_pmc.sh writes them under gpurun_out/pmc/, one
directory per (config, pass): <config>_fetch, <config>_write, <config>_core).

Per config and kernel role -- the decoder heads launch, the per-image fp-half
store launch, the correlation launch -- the per-launch FETCH_SIZE (raw and
x2-corrected) and WRITE_SIZE bytes, the core counters, MFMA busy and the
effective clock (pmc_csv.py).  bench.py reads the record of the config it
runs (and only when the run uses the config's own options): `traffic` of its
roofline objects is that record's hbm_bytes_per_launch, or null.

    python profiles/pmc_assemble.py <pmc-dir> <round-label> [out.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_csv import summarize  # noqa: E402


def _buildinfo():
    """tmr_amd/buildinfo.py loaded by path (no torch, no package import)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "template-matching-and-regression-mapreduce_amd", "buildinfo.py")
    spec = importlib.util.spec_from_file_location("tmr_buildinfo", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod

# role -> kernel regex (rocprofv3 CSV names are demangled for the split and
# rows kernels, mangled for the MFMA correlation)
ROLES = {
    "heads": r"split_conv_kernel<\d+, \d+, 1>",
    "store": r"split_conv_kernel<[3-7], \d+, 0>",
    "xcorr": r"xcorr_(rows|mfma)_kernel",
}
CONFIGS = ("A", "B", "C", "D", "E")


def main(pmc_dir, label, out):
    res = {"note": ("rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE and the SQ/GRBM group in "
                    "separate runs) of `python bench.py --config <c> --steps 1 --warmup 0 "
                    "--no-cpu-baseline --no-xcorr-classes` (profiles/gpu_pmc.sh, round %s): one "
                    "launch per role in each run. Per launch of the role's largest grid: "
                    "fetch_bytes_x2 = 2 x FETCH_SIZE (gfx950 reports 1/2 of 16-B/lane streaming "
                    "reads, MI355X_MICROARCH.md HBM), hbm_bytes_per_launch = fetch_bytes_x2 + "
                    "write_bytes. FETCH_SIZE counts Infinity-Cache hits too: it is traffic beyond "
                    "L2, an upper bound of HBM bytes. mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / "
                    "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)." % label),
           "round": label, "configs": {}}
    for cfg in CONFIGS:
        passes = [os.path.join(pmc_dir, f"{cfg}_{p}") for p in ("fetch", "write", "core")]
        dirs = [d for d in passes if os.path.isdir(d)]
        if not dirs:
            continue
        rec = {}
        for role, kern in ROLES.items():
            r = summarize(kern, dirs)
            if "fetch_bytes_raw" not in r and "write_bytes" not in r:
                continue
            r.pop("launches", None)
            c = r["counters"]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
                r["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
            # the tree the counters belong to: bench.py prints them only
            # while the kernel's sources are unchanged
            r["source_digest"] = _buildinfo().source_digest(role)
            rec[role] = r
        res["configs"][cfg] = rec
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({c: {r: (v.get("avg_launch_s"), v.get("hbm_bytes_per_launch"))
                          for r, v in rec.items()} for c, rec in res["configs"].items()}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else
         os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_by_config.json"))
