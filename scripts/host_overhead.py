"""Host-side overhead of one bench step (reset + rollout) next to the device time."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdcommunity_amd import _lib, engine, gmm
e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
e.load_graphs([(1000,) + gmm.gmm_pair(1000, seed=0)])
for _ in range(3):
    e.reset(); e.rollout()
R = []
for _ in range(10):
    t0 = time.perf_counter(); e.reset(); t1 = time.perf_counter(); k0 = e.last_timing()[0]
    e.rollout(); t2 = time.perf_counter(); k1 = e.last_timing()[0]
    R.append(((t1 - t0) * 1e3, k0, (t2 - t1) * 1e3, k1))
R = np.median(np.array(R), axis=0)
print("reset wall %.3f ms (kernel %.3f) | rollout wall %.3f ms (kernel %.3f) | host overhead %.3f ms" % (
    R[0], R[1], R[2], R[3], R[0] - R[1] + R[2] - R[3]))
