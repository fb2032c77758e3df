"""Useful-FLOP table of the depthwise correlation's Toeplitz formulations on
each 16-bit gfx950 MFMA shape: per template side w (h = w),
the useful share of each instruction's MACs times the shape's measured FLOP
rate (profiles/mfma_shapes/results/mfma_shapes16.jsonl: random fp16 operands,
16 independent accumulator chains per wave, 2 waves per SIMD on every CU).

Row forms (round 5 and the alternatives): M output columns of one row against
a K-wide input window per template row; the window must hold M + w - 1
columns, so a row takes ceil((M + w - 1) / K) K-blocks and the useful share
is w / (K * blocks).  2-D window form (round 6, xcorr_mfma_kernel): M = 16
outputs as 2 rows x 8 columns against K = 32 inputs as 4 rows x 8 columns,
ceil((h + 1) / 4) x ceil((w + 7 + s) / 8) windows with s = (-(w // 2)) mod 8
(16-B aligned LDS reads): useful share h w / (32 windows).

    python profiles/mfma_shapes/toeplitz.py > profiles/mfma_shapes/toeplitz_table.md
"""
import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))
RATE = {json.loads(l)["shape"]: json.loads(l)["tflops"]
        for l in open(os.path.join(HERE, "results", "mfma_shapes16.jsonl")) if l.startswith("{")}

# (label, measured shape, M outputs per block row, K inputs per block)
ROW_FORMS = [
    ("row 16x16x32 (round 5)", "f16_16x16x32", 16, 32),
    ("row 16x16x16", "f16_16x16x16", 16, 16),
    ("row 32x32x16", "f16_32x32x16", 32, 16),
    ("row 32x32x8", "f16_32x32x8", 32, 8),
    ("row 16x16x4 (4 blocks)", "f16_16x16x4_4b", 16, 4),
    ("row 4x4x4 (16 blocks)", "f16_4x4x4_16b", 4, 4),
]


def row_useful(w, m, k):
    return w / (k * math.ceil((m + w - 1) / k))


def window_useful(w, h=None):
    h = w if h is None else h
    s = (-(w // 2)) % 8
    return h * w / (32 * math.ceil((h + 1) / 4) * math.ceil((w + 7 + s) / 8))


def main():
    ws = list(range(3, 32, 2))
    cols = [(lbl, RATE[shape], (lambda w, m=m, k=k: row_useful(w, m, k))) for lbl, shape, m, k in ROW_FORMS]
    cols.insert(1, ("2-D window 16x16x32 (round 6)", RATE["f16_16x16x32"], window_useful))
    print("# Useful TFLOP/s by formulation (useful share x measured shape rate)\n")
    print("Measured rates (TFLOP/s, fp16, random operands): "
          + ", ".join(f"{s} {r:.0f}" for s, r in RATE.items() if s.startswith("f16")) + "\n")
    print("| w | " + " | ".join(c[0] for c in cols) + " |")
    print("|---:|" + "---:|" * len(cols))
    for w in ws:
        print(f"| {w} | " + " | ".join(f"{f(w):.2f} x {r:.0f} = **{f(w) * r:.0f}**" for _, r, f in cols) + " |")


if __name__ == "__main__":
    main()
