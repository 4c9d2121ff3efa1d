import os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from mdcommunity_amd import _lib, engine, synth, agent
n = 18000
layers = synth.real_like_layers(n, 0)
es = []
for lay in layers:
    seen, order = set(), []
    for u, v in lay:
        k = (min(u, v), max(u, v))
        if u != v and k not in seen:
            seen.add(k); order.append(k)
    es.append(np.array(order, np.int32))
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT_REAL))
eng.load_graphs([(n, es[0], es[1])])
eng.reset()
for t in range(8):
    q, am, nt, gap = eng.predict()
    pm, pl = eng.last_timing()
    a = int(np.argmax(np.where(np.isfinite(q), q, -np.inf)))
    lm, term = eng.step(np.array([a], np.int32))
    sm, sl = eng.last_timing()
    print(f"step {t}: predict {pm*1e3:.0f} us ({pl} launches), env step {sm*1e3:.0f} us, lmcc {lm[0]}, live {np.isfinite(q).sum()}", flush=True)
