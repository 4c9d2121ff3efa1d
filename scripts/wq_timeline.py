"""Per-step timeline of the first graph slot (the most edges: the longest rollout) in one wave-item
batch launch (md_wq_kernel event log, MD_VARIANT bit 4): environment step, the three tile stages
and the virtual node, in microseconds.
  MD_PROF_ALL=1 MD_VARIANT=$((256*65536+4)) MD_WQPARK=0 python scripts/wq_timeline.py [graphs]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm_gpu
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
W = engine.load_weights(engine.DEFAULT_UNIT)
graphs = [(1000,) + e for e in gmm_gpu.gmm_pairs(1000, range(nb), exact=True)]
eng = _lib.Engine(W)
eng.load_graphs(graphs)
eng.reset(); eng.rollout()
eng.reset()
eng.profile(64)
eng.rollout()
ms, launches = eng.last_timing()
P = eng.profile_read(64).astype(np.int64).reshape(-1)
eng.profile(0)
n = int(P[8 * 96 - 1])
ev = P[8 * 96: 8 * 96 + 2 * n].reshape(-1, 2)
t0 = ev[0, 1]
names = {0: "ENV", 1: "st1", 2: "st2", 3: "st3", 4: "VN2"}
print(f"batch {nb}: kernel {ms:.2f} ms, {launches} launches, {n} events of graph slot 0")
# per step: ENV taken (6) -> group start (0) -> tiles pushed (5) -> st1 -> st2 -> VN2 -> st3
steps, cur = [], {}
for e, t in ev:
    e = int(e)
    if e == 6:
        if cur:
            steps.append(cur)
        cur = {6: t}
    else:
        cur.setdefault(e, t)
if cur:
    steps.append(cur)
order = (6, 0, 5, 1, 2, 4, 3)
labels = ("rendezvous", "ENV", "->it1 done", "it2", "VN2", "it3", "->next ENV taken")
d = []
for i, s in enumerate(steps):
    if all(k in s for k in order) and i + 1 < len(steps):
        ts = [s[k] for k in order] + [steps[i + 1][6]]
        d.append(np.diff(ts))
d = np.asarray(d) / 100.0
if len(d):
    print("steps with a forward pass: %d; median us: " % len(d) +
          ", ".join("%s %.1f" % (l, v) for l, v in zip(labels, np.median(d, axis=0))) +
          "; total %.1f" % np.median(d.sum(axis=1)))
    print("mean us: " + " ".join("%.1f" % x for x in d.mean(axis=0)))
print("graph slot 0 span %.2f ms over %d steps" % ((ev[-1, 1] - t0) / 1e5, len(steps)))
eng.close()
