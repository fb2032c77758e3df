"""Why does (or doesn't) TMREngine.detect capture its forward?  Calls detect
three times on one signature and prints which signature components differ
between calls, the graph mode of each call and any capture error."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

tmr = load_package()
from tmr_amd import host, synth  # noqa: E402

dev = torch.device("cuda:0")
cin, emb, hf, B, E = 32, 64, 16, 2, 3
P = {k: v.to(dev) for k, v in synth.reference_state_dict(12, cin=cin, emb=emb, obj_bias=0.4).items()}
eng = tmr.TMREngine(P, tmr.PathConfig(emb_dim=emb))
ex, _ = synth.exemplar_set(40, B, E, 2 * hf, 2 * hf, 3, 7)
feats = torch.from_numpy(synth.sam_features(41, B, cin, hf, hf)).to(dev)
ui = np.repeat(np.arange(B), E)
sigs = []
for i in range(4):
    units = host.build_units(ex.reshape(-1, 4), ui, 2 * hf, 2 * hf, emb)[0]
    sigs.append(eng._graph_signature(feats, units, ui, False, False))
    eng.detect(feats, ex, 0.5, 0.5)
    print(i, eng.last_graph, eng.last_graph_error, list(eng._graph_seen.values()), flush=True)
for i in range(1, len(sigs)):
    if sigs[i] is None or sigs[0] is None:
        print("sig None", i)
        continue
    diff = [j for j, (a, b) in enumerate(zip(sigs[0], sigs[i])) if a != b]
    print("call", i, "differs from call 0 in components", diff)
    for j in diff:
        print("  ", j, str(sigs[0][j])[:300], "->", str(sigs[i][j])[:300])
