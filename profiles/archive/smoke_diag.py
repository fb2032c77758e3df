"""Smoke-input survey: kept boxes and GPU-vs-oracle set agreement for a few
objectness biases / thresholds (near-tied scores reorder NMS when the score
maps differ in the last ulp)."""
import os, sys
import numpy as np, torch
REPO = os.getcwd()
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
from tmr_import import load_package
tmr = load_package()
import oracle
dev = torch.device("cuda:0")
feats = tmr.synth.sam_features(1, 2, 32, 16, 16)
ex, _ = tmr.synth.exemplar_set(2, 2, 3, 32, 32, 3, 7)
for bias, cls in [(0.5, 0.5), (0.0, 0.5), (0.0, 0.502), (-1.0, 0.2689), (0.5, 0.623)]:
    P = oracle.reference_weights(0, cin=32, emb=32)
    P["objectness_head.head.0.bias"] = torch.tensor([bias])
    eng = tmr.TMREngine({k: v.to(dev) for k, v in P.items()}, tmr.PathConfig(emb_dim=32))
    L, Bx, R = eng.detect(torch.from_numpy(feats).to(dev), ex, cls_ths=cls, iou_threshold=0.5)
    torch.cuda.synchronize()
    out = []
    for b in range(2):
        ls, bs, rs = [], [], []
        for e in range(3):
            exm = [torch.from_numpy(ex[b, e:e + 1])]
            o, bb, _, _ = oracle.forward_torch(torch.from_numpy(feats[b:b + 1]), exm, P)
            prob = oracle.sigmoid_cr(o[0][0, 0].numpy())
            l_, b_, r_ = oracle.get_pred_boxes_prob([prob], [bb[0][0].numpy()], exm, cls)
            ls.append(l_[0]); bs.append(b_[0]); rs.append(r_[0])
        lo, bo, ro = oracle.nms_lists([np.concatenate(ls)], [np.concatenate(bs)], [np.concatenate(rs)], 0.5)
        got, exp = Bx[b].cpu().numpy(), bo[0]
        nb = -1
        if got.shape == exp.shape and got.size:
            d = np.abs(got[:, None, :] - exp[None, :, :]).max(-1)
            nb = int((d.min(1) > 1e-4).sum())
        ordered = got.shape == exp.shape and np.allclose(got, exp, rtol=1e-4, atol=1e-5)
        out.append((got.shape[0], exp.shape[0], nb, ordered))
    print("bias", bias, "cls", cls, out, flush=True)
