"""Paired-tile debugging: per-prediction max Q of queue-mode rollouts with MD_PAIR=0 and 1
(admission 1, two tiles per item), printed side by side up to the first difference."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden
from mdcommunity_amd import _lib, engine

names = ["gmm200_s7", "er100", "er300_dense"]
graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
os.environ["MD_VARIANT"] = str((1 << 16) | (2 << 9))
res = {}
for pair in ("0", "1"):
    os.environ["MD_PAIR"] = pair
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    e.load_graphs([graphs[i % 3] for i in range(18)])
    e.reset()
    out = e.rollout()
    res[pair] = (out, [e.trace(g) for g in range(3)])
    e.close()
for g in range(3):
    a, b = res["0"][1][g], res["1"][1][g]
    sa, sb = res["0"][0][g][0], res["1"][0][g][0]
    print(names[g], "seq equal", np.array_equal(sa, sb), "len", len(sa), len(sb))
    k = min(len(a["qmax"]), len(b["qmax"]))
    for t in range(k):
        d = float(a["qmax"][t]) - float(b["qmax"][t])
        print("  pred %2d n_live %4d/%4d qmax %.9g / %.9g diff %.3g" % (t, a["n_live"][t], b["n_live"][t], a["qmax"][t], b["qmax"][t], d))
        if d != 0 and t > 3:
            break
