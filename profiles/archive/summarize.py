"""Summarise a rocprofv3 kernel-trace database (run_results.db) into the
per-kernel table committed under profiles/ (calls, total, average, share).

    python profiles/summarize.py gpurun_out/prof_r1a/run_results.db > profiles/archive/r01_kernel_stats.md
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, total_calls, total_duration, average, percentage "
                     "from top_kernels order by total_duration desc").fetchall()
    meta = dict(c.execute("select tag, value from rocpd_metadata").fetchall()) \
        if c.execute("select count(*) from sqlite_master where name='rocpd_metadata'").fetchone()[0] \
        else {}
    print(f"# rocprofv3 --kernel-trace --stats summary ({path.split('/')[-2]})\n")
    if meta:
        print("metadata: " + ", ".join(f"{k}={v}" for k, v in sorted(meta.items())[:6]) + "\n")
    print("| kernel | calls | total (us) | average (us) | % |")
    print("|---|---:|---:|---:|---:|")
    for name, n, tot, avg, pct in rows:
        short = name if len(name) < 110 else name[:107] + "..."
        print(f"| `{short}` | {n} | {tot:.1f} | {avg:.1f} | {pct:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
