"""Host checks of integer/float identities the HIP kernels rely on (no GPU).

xcorr.hip (xcorr_rows_kernel staging) computes the band row of float4 slot e
as (int)(((float)e + 0.5f) * (1.0f / WS4)) instead of e / WS4.  Every fp32
operation there is a single IEEE round-to-nearest (the Makefile builds with
-ffp-contract=off), so numpy float32 arithmetic reproduces it exactly.
"""
import numpy as np


def test_xcorr_band_row_index_by_reciprocal_is_exact():
    # slots per band stay below 2^16 (LDS <= 160 KB = 10240 float4); row
    # widths WS4 = W/4 + 11 for every W % 4 == 0 up to 4356 columns
    e = np.arange(1 << 16, dtype=np.int64)
    ef = e.astype(np.float32) + np.float32(0.5)
    for ws4 in range(11, 1100):
        r = np.float32(1.0) / np.float32(ws4)
        q = (ef * r).astype(np.float32)
        assert np.array_equal(q.astype(np.int64), e // ws4), ws4
