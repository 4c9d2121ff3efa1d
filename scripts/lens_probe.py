import sys, numpy as np
sys.path.insert(0, "/root/repo")
from mdcommunity_amd import _lib, engine, gmm
W = engine.load_weights(engine.DEFAULT_UNIT)
gs = [(1000,) + gmm.gmm_pair(1000, seed=s) for s in range(256)]
e = _lib.Engine(W); e.load_graphs(gs); mr = e.reset(); out = e.rollout()
lens = np.array([len(o[0]) for o in out])
E = np.array([len(g[1]) + len(g[2]) for g in gs])
np.savez("gpurun_out/lens.npz", lens=lens, mr=np.asarray(mr), E=E)
print(np.corrcoef(lens, mr)[0,1], np.corrcoef(lens, E)[0,1])
