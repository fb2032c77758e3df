"""TEST INFRASTRUCTURE ONLY -- golden vectors for the streaming reducer.

Runs the reference's own reducer.py (/root/reference/reducer.py, a stdin ->
stdout/stderr program) on seeded synthetic mapper output and stores
{input lines, stdout, stderr} per case in tests/golden/reducer_cases.json.
Cases: the Hadoop-sorted output of mapper-format lines over the three RPINE
categories; interleaved categories (the reducer groups consecutive keys
only); malformed lines (no tab, 4 values, non-numeric); a zero-count
category (division error path); > 100 lines (progress messages); empty
input.  Nothing from the reference is copied; only its output is stored.

Usage (this container only; /root/reference is absent on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python oracle/make_golden_stream.py
"""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference/reducer.py"
sys.path.insert(0, HERE)
import oracle  # noqa: E402


def run_ref(lines):
    p = subprocess.run([sys.executable, REF], input="".join(l + "\n" for l in lines),
                       capture_output=True, text=True, env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"),
                       check=True)
    return p.stdout, p.stderr


def mapper_lines(rng, shards):
    out = []
    for name in shards:
        cat = name.split("_")[0]
        n = rng.randint(3, 6)
        stats = [(rng.gauss(0, 0.01), rng.uniform(0.9, 1.1), rng.uniform(3, 8), rng.uniform(0.4, 0.6))
                 for _ in range(n)]
        stats = [tuple(float(__import__("numpy").float32(v)) for v in s) for s in stats]
        sums, cnt = oracle.mapper_tar_sums(stats)
        out.append(oracle.mapper_line(cat, sums, cnt))
    return out


def main():
    rng = random.Random(7)
    shards = [f"{c}_{i}.tar" for c in ("Easy", "Normal", "Hard") for i in range(40)]
    rng.shuffle(shards)
    lines = mapper_lines(rng, shards)
    cases = {}
    cases["sorted"] = sorted(lines, key=lambda l: l.split("\t")[0])  # Hadoop shuffle
    cases["interleaved"] = lines[:12]
    bad = sorted(lines[:20], key=lambda l: l.split("\t")[0])
    bad[3:3] = ["Easy 1,2,3,4,5", "Easy\t1,2,3,4", "Hard\tx,1,2,3,4", "", "Normal\t1,2,3,4,5,6",
                "Normal\t0.1,0.2,0.3,0.4,2.5"]
    cases["malformed"] = bad
    cases["zero_count"] = ["Easy\t0.0,0.0,0.0,0.0,0", "Easy\t0.0,0.0,0.0,0.0,0",
                           "Hard\t0.5,1.0,4.0,0.5,1"]
    many = [l for l in lines for _ in range(2)][:230]
    cases["progress"] = sorted(many, key=lambda l: l.split("\t")[0])
    cases["empty"] = []
    out = {}
    for k, v in cases.items():
        so, se = run_ref(v)
        out[k] = {"input": v, "stdout": so, "stderr": se}
    dst = os.path.join(REPO, "tests", "golden", "reducer_cases.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", dst, {k: len(v["input"]) for k, v in out.items()})


if __name__ == "__main__":
    main()
