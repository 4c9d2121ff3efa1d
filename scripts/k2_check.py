import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from mdcommunity_amd import _lib, engine, gmm
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
bad = tot = k2 = 0
for s in range(40):
    e = gmm.gmm_pair(1000, seed=s)
    eng.load_graphs([(1000,) + e])
    eng.reset(); eng.rollout()
    tr = eng.trace(0)
    for nl, m0, m1, nt in zip(tr["n_live"], tr["m0"], tr["m1"], tr["n_tie"]):
        tot += 1
        if 2 * m0 == nl and 2 * m1 == nl:
            k2 += 1
            if nt != nl:
                bad += 1
print("steps", tot, "all-K2 states", k2, "of which not all tied", bad)
