"""Assemble profiles/decoder_pmc.json from one measurement round's rocprofv3
--pmc passes (profiles/gpu_round.sh writes them under gpurun_out/pmc/):
per kernel variant the per-launch FETCH_SIZE (raw and x2-corrected) and
WRITE_SIZE bytes, the core counters and the effective clock (pmc_csv.py).

    python profiles/pmc_assemble.py <pmc-dir> <round-label> [out.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_csv import summarize  # noqa: E402

# variant -> (kernel substring, passes)
VARIANTS = {
    "split_fp32": ("split_conv_kernel<3, 0, 1>", ["B_fetch", "B_write", "B_core"]),
    "split_fp32_store": ("split_conv_kernel<3, 0, 0>", ["B_fetch", "B_write", "B_core"]),
    "split_bf16": ("split_conv_kernel<3, 1, 1>", ["C_fetch", "C_write"]),
    "xcorr": ("xcorr_rows_kernel", ["B_fetch", "B_write", "B_core"]),
}
ALG = ("Algorithmic bytes per heads launch (192 units): f_TM records 192 x 34.6 MB + acc0 192 x "
       "134.2 MB + weights 37.7 MB + head partials 192 x 5.2 MB = 33.5 GB; the excess is weight "
       "and halo re-reads by the 16 channel tiles and the 32 pixel tiles, served from Infinity Cache.")


def main(pmc_dir, label, out):
    res = {"note": ("rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE and the SQ/GRBM group in "
                    "separate runs) of `python bench.py --steps 1 --warmup 0 --no-cpu-baseline "
                    "[--config C]` (profiles/gpu_round.sh, round %s). Per launch of the kernel's "
                    "main grid: fetch_bytes_x2 = 2 x FETCH_SIZE (gfx950 reports 1/2 of 16-B/lane "
                    "streaming reads, MI355X_MICROARCH.md HBM), hbm_bytes_per_launch = "
                    "fetch_bytes_x2 + write_bytes. FETCH_SIZE counts Infinity-Cache hits too: it "
                    "is traffic beyond L2, an upper bound of HBM bytes. " % label) + ALG}
    for name, (kern, passes) in VARIANTS.items():
        dirs = [os.path.join(pmc_dir, p) for p in passes if os.path.isdir(os.path.join(pmc_dir, p))]
        if not dirs:
            continue
        r = summarize(kern, dirs)
        if "fetch_bytes_raw" not in r:
            continue
        r.pop("launches", None)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in r["counters"] and "SQ_BUSY_CYCLES" in r["counters"]:
            # MFMA pipe busy fraction: busy cycles over 1024 SIMDs x the per-XCD GPU cycles
            c = r["counters"]
            r["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        res[name] = r
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: (v.get("avg_launch_s"), v.get("hbm_bytes_per_launch")) for k, v in res.items()
                      if isinstance(v, dict)}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else
         os.path.join(os.path.dirname(os.path.abspath(__file__)), "decoder_pmc.json"))
