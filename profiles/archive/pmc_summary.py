"""Summarise rocprofv3 --pmc passes (one counter set per pass, separate runs)
for one kernel into JSON: per-launch FETCH_SIZE / WRITE_SIZE bytes and L2 hit
rate.  MI355X_MICROARCH.md (HBM): FETCH_SIZE = TCC_EA0_RDREQ x 64 B counts
Infinity-Cache hits too and reports 1/2 of the bytes of 16-B-per-lane
streaming reads; other widths are uncalibrated.  We report the raw counter and
the x2-corrected upper bound.

    python profiles/pmc_summary.py <kernel-substring> <algorithmic_bytes> <out.json> <db>...
"""
import json
import sqlite3
import sys


def main(kernel, alg_bytes, out, dbs):
    vals = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, counter, value in c.execute(
                "select kernel_name, counter_name, value from counters_collection"):
            if kernel in name:
                vals.setdefault(counter, []).append(float(value))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {"kernel": kernel, "launches": {k: len(v) for k, v in vals.items()},
           "algorithmic_bytes_per_launch": alg_bytes}
    if "FETCH_SIZE" in avg:
        res["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
        res["fetch_bytes_x2_upper"] = 2 * res["fetch_bytes_raw"]
    if "WRITE_SIZE" in avg:
        res["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        res["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "fetch_bytes_raw" in res and "write_bytes" in res:
        res["hbm_bytes_per_launch"] = res["fetch_bytes_raw"] + res["write_bytes"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4:])
