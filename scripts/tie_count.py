import os, sys, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mdcommunity_amd import _lib, engine, gmm
e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
e.load_graphs([(1000,) + gmm.gmm_pair(1000, seed=0)])
for _ in range(3):
    e.reset(); e.rollout()
e.reset(); e.rollout()
tr = e.trace(0)
nt = np.asarray(tr["n_tie"])
print("predictions", len(nt), "ties>1 at", np.flatnonzero(nt > 1).tolist(), "kernel ms", e.last_timing()[0], flush=True)
