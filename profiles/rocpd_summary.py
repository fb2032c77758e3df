"""Kernel-time summary of a rocprofv3 --kernel-trace run from its rocpd
SQLite output (<dir>/**/*results.db; rocprofv3's default output format on the
GPU boxes) or its CSV (*kernel_trace.csv): the per-kernel stats table
(markdown) and, per bench step, GPU busy time (union of kernel intervals)
against the step's span, i.e. the idle time the host leaves between
launches.  Steps are delimited by the launches of `--step-kernel` (one per
bench step, default: the decoder heads launch).

    python profiles/rocpd_summary.py <dir> [--label L] [--step-kernel REGEX]
"""
import argparse
import collections
import csv
import glob
import os
import re
import sqlite3


def load(d):
    rows = []
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        for name, start, end in con.execute("select name, start, end from kernels"):
            rows.append((name, int(start), int(end)))
    if not rows:
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(rows, key=lambda r: r[1])


def busy(iv):
    t, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                t += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        t += cur_e - cur_s
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--label", default=None)
    ap.add_argument("--step-kernel", default=r"split_conv_kernel<\d+, \d+, 1>")
    a = ap.parse_args()
    rows = load(a.dir)
    tot = collections.defaultdict(lambda: [0, 0])
    for n, s, e in rows:
        tot[n][0] += 1
        tot[n][1] += e - s
    all_t = sum(v[1] for v in tot.values())
    print(f"# rocprofv3 --kernel-trace summary ({a.label or os.path.basename(a.dir.rstrip('/'))})\n")
    print("| kernel | calls | total (us) | average (us) | % |\n|---|---:|---:|---:|---:|")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        nm = n if len(n) <= 110 else n[:107] + "..."
        print(f"| `{nm}` | {c} | {t / 1e3:.1f} | {t / c / 1e3:.1f} | {100 * t / all_t:.2f} |")
    pat = re.compile(a.step_kernel)
    marks = [s for n, s, _ in rows if pat.search(n)]
    if len(marks) >= 2:
        print("\n## Per bench step (from one step-kernel launch to the next)\n")
        print("| step | span (ms) | GPU busy (ms) | idle (ms) | idle % |\n|---:|---:|---:|---:|---:|")
        for i in range(len(marks) - 1):
            s0, s1 = marks[i], marks[i + 1]
            iv = [(max(s, s0), min(e, s1)) for _, s, e in rows if e > s0 and s < s1]
            b = busy(iv)
            print(f"| {i} | {(s1 - s0) / 1e6:.3f} | {b / 1e6:.3f} | {(s1 - s0 - b) / 1e6:.3f} | "
                  f"{100 * (s1 - s0 - b) / (s1 - s0):.1f} |")


if __name__ == "__main__":
    main()
