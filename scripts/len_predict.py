"""How well do a graph's reset-time figures predict its rollout length?  (C3 batch: 256 GMM
N=1000 graphs.)  Prints the rank correlation of the length with max_rank and with the edge
count, and how many of the longest rollouts a top-k pick by each figure catches.
  python scripts/len_predict.py [graphs]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm_gpu
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
W = engine.load_weights(engine.DEFAULT_UNIT)
pairs = gmm_gpu.gmm_pairs(1000, range(nb), exact=True)
graphs = [(1000,) + e for e in pairs]
eng = _lib.Engine(W)
eng.load_graphs(graphs)
mr = eng.reset().astype(np.int64)
out = eng.rollout()
L = np.array([len(o[0]) for o in out])
E = np.array([len(e0) + len(e1) for e0, e1 in pairs])
R1 = np.array([int(o[1][0]) if len(o[1]) else 0 for o in out])  # LMCC after the first removal
eng.close()


def rk(x):
    return np.argsort(np.argsort(x, kind="stable"), kind="stable").astype(np.float64)


def spear(a, b):
    return float(np.corrcoef(rk(a), rk(b))[0, 1])


print("lengths min/median/max %d/%d/%d, sum %d" % (L.min(), np.median(L), L.max(), L.sum()))
for name, x in (("max_rank", mr), ("edges", E), ("rank after step 1", R1)):
    print("%-18s spearman %.3f" % (name, spear(x, L)))
    for frac in (0.1, 0.25):
        k = max(1, int(frac * nb))
        top_len = set(np.argsort(-L, kind="stable")[:k].tolist())
        top_x = set(np.argsort(-x, kind="stable")[:k].tolist())
        pick = np.argsort(-x, kind="stable")[:k]
        print("   top %2d%%: %d of the %d longest caught; shortest picked %d; longest missed %d" % (
            int(frac * 100), len(top_len & top_x), k, L[pick].min(),
            max([L[i] for i in top_len - top_x], default=0)))
