"""Small batches (the k longest rollouts of the C3 batch) in the lock-step kernel with and
without the solo hand-off (MD_SOLO): kernel ms per batch rollout."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm_gpu
W = engine.load_weights(engine.DEFAULT_UNIT)
graphs = [(1000,) + e for e in gmm_gpu.gmm_pairs(1000, range(64), exact=True)]
e = _lib.Engine(W)
e.load_graphs(graphs); e.reset(); out = e.rollout(); e.close()
lens = np.array([len(o[0]) for o in out])
order = np.argsort(-lens, kind="stable")
for k in (2, 4, 8, 16):
    row = []
    for solo in ("0", "1"):
        os.environ["MD_SOLO"] = solo
        e = _lib.Engine(W)
        e.load_graphs([graphs[i] for i in order[:k]])
        e.reset(); e.rollout()
        ts = []
        for _ in range(5):
            e.reset(); e.rollout(); ts.append(e.last_timing())
        e.close()
        ts.sort()
        row.append(ts[2])
    print("longest %2d: MD_SOLO=0 %.2f ms (%d launches), MD_SOLO=1 %.2f ms (%d launches)" % (k, row[0][0], row[0][1], row[1][0], row[1][1]), flush=True)
