"""Host-side time around the headline rollout (bench.py run_steps): reset_deferred, rollout
(split into device kernel time and the rest), max_rank -- medians over repeated steps.
  python scripts/host_overhead.py [reps]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
z = np.load(os.path.join(ROOT, "tests/golden/rollout_gmm1000_s0.npz"))
e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
T = []
for i in range(reps + 3):
    t0 = time.perf_counter()
    e.reset_deferred()
    t1 = time.perf_counter()
    outs = e.rollout()
    t2 = time.perf_counter()
    ms, nl = e.last_timing()
    mr = e.max_rank()
    t3 = time.perf_counter()
    if i >= 3:
        T.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, ms, (t3 - t2) * 1e3, (t3 - t0) * 1e3))
T = np.array(T)
m = np.median(T, axis=0)
print("median ms: reset_deferred %.3f  rollout %.3f (kernel %.3f, rest %.3f)  timing+max_rank %.3f  step %.3f" % (
    m[0], m[1], m[2], m[1] - m[2], m[3], m[4]))
e.close()
