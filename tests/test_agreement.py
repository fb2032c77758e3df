"""The end-to-end detection contract between two fp32 runs of the same forward
(oracle/agreement.py), measured on the REFERENCE ITSELF: the CPU oracle's
forward at 1 thread vs all threads (ATen's summation order changes with the
thread count, SURVEY.md §4: 9e-7 normwise) on the smoke input with dense,
near-tied candidates (objectness bias 0.5).  CPU only."""
import os

import numpy as np
import torch

import agreement
import oracle
from tmr_amd import synth


def _maps(P, feats, ex, nt):
    torch.set_num_threads(nt)
    out = []
    for b in range(feats.shape[0]):
        m = []
        for e in range(ex.shape[1]):
            o, bb, _, _ = oracle.forward_torch(torch.from_numpy(feats[b:b + 1]),
                                               [torch.from_numpy(ex[b, e:e + 1])], P)
            m.append((oracle.sigmoid_cr(o[0][0, 0].numpy()), bb[0][0].numpy()))
        out.append(m)
    return out


def test_reference_thread_count_detection_noise():
    nt0 = torch.get_num_threads()
    try:
        P = oracle.reference_weights(0, cin=32, emb=32)
        P["objectness_head.head.0.bias"] = torch.tensor([0.5])
        feats = synth.sam_features(1, 2, 32, 16, 16)
        ex, _ = synth.exemplar_set(2, 2, 3, 32, 32, 3, 7)
        m1 = _maps(P, feats, ex, 1)
        mn = _maps(P, feats, ex, max(2, min(8, os.cpu_count() or 2)))
    finally:
        torch.set_num_threads(nt0)
    for b in range(2):
        rep = agreement.compare(m1[b], mn[b], list(ex[b]), 0.5, 0.5)
        print(agreement.report_line(f"reference 1 vs N threads, image {b}:", rep))
        agreement.check(rep)
        assert rep["max_dprob"] <= 1e-6
        assert rep["matched_iou_mean"] > 0.99
    # the same run against itself: no flip, identical
    rep = agreement.compare(m1[0], m1[0], list(ex[0]), 0.5, 0.5)
    assert rep["flips"] == 0 and rep["same_kept_ids"] and rep["kept_box_max_diff"] == 0.0
