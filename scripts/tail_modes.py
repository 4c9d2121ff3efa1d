"""The launch tail: the k longest rollouts of the C3 batch run as their own batch in the
lock-step kernel (dedicated environment workgroups, <= 16 graphs) and in queue mode
(MD_ENV_MODE=0), kernel ms each -- what a queue launch that hands its last graphs to the
lock-step kernel could save."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm_gpu
W = engine.load_weights(engine.DEFAULT_UNIT)
graphs = [(1000,) + e for e in gmm_gpu.gmm_pairs(1000, range(256), exact=True)]
e = _lib.Engine(W)
e.load_graphs(graphs); e.reset(); out = e.rollout(); e.close()
lens = np.array([len(o[0]) for o in out])
order = np.argsort(-lens, kind="stable")
for k in (1, 4, 8, 16):
    sel = [graphs[i] for i in order[:k]]
    row = []
    for env_mode in ("1", "0"):
        os.environ["MD_ENV_MODE"] = env_mode
        e = _lib.Engine(W)
        e.load_graphs(sel)
        e.reset(); e.rollout()
        ts = []
        for _ in range(5):
            e.reset(); e.rollout(); ts.append(e.last_timing()[0])
        e.close()
        row.append(min(ts))
    print("longest %2d (lengths %s): lock-step %.2f ms, queue %.2f ms" % (k, lens[order[:k]].tolist()[:4], row[0], row[1]), flush=True)
