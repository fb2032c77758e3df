"""Per-launch averages of rocprofv3 --pmc counters (CSV output, one counter
set per pass/run) for the kernels whose name matches a regular expression
(a plain substring works as one).

    python profiles/pmc_csv.py <kernel-regex> <dir-or-csv>...

Prints {counter: mean per launch} plus launch counts as JSON.  HBM byte
conventions (MI355X_MICROARCH.md, HBM): FETCH_SIZE / WRITE_SIZE are in KB;
FETCH_SIZE reports 1/2 of the bytes of 16-B-per-lane streaming reads (the
x2-corrected value is reported beside the raw one); effective clock =
GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def collect(kernel, paths):
    """Counter values and durations of the matching launches with the
    largest grid (a kernel's small side launches, e.g. the one-off bias-plane
    launch of split_conv_kernel<3,0,0>, are left out of the averages)."""
    rows = []
    pat = re.compile(kernel)
    for p in paths:
        files = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True) \
            if os.path.isdir(p) else [p]
        for f in files:
            for row in csv.DictReader(open(f)):
                if pat.search(row["Kernel_Name"]):
                    rows.append((f, row))
    gmax = max((int(r["Grid_Size"]) for _, r in rows), default=0)
    vals = collections.defaultdict(list)
    dur = []
    seen = set()
    names = set()
    for f, row in rows:
        if int(row["Grid_Size"]) != gmax:
            continue
        names.add(row["Kernel_Name"])
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        key = (f, row["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    collect.names = sorted(names)
    return vals, dur


def summarize(kernel, paths):
    vals, dur = collect(kernel, paths)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {"kernel": kernel, "kernel_names": getattr(collect, "names", []),
           "launches": {k: len(v) for k, v in vals.items()}, "counters": avg}
    if dur:
        res["avg_launch_s"] = sum(dur) / len(dur)
    if "FETCH_SIZE" in avg:
        res["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
        res["fetch_bytes_x2"] = 2 * res["fetch_bytes_raw"]
    if "WRITE_SIZE" in avg:
        res["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "fetch_bytes_x2" in res and "write_bytes" in res:
        res["hbm_bytes_per_launch"] = res["fetch_bytes_x2"] + res["write_bytes"]
    if "GRBM_GUI_ACTIVE" in avg and dur:
        res["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / res["avg_launch_s"] / 1e9
    return res


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1], sys.argv[2:]), indent=1))
