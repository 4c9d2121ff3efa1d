"""Queue-mode admission order experiment: the same 256 graphs loaded in seed order, in
descending edge count, and in descending rollout length (known from a first run: the ideal
longest-first bound).  Per-graph results do not depend on the order; the launch time does
through the tail (the longest rollouts admitted last run alone)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm_gpu

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
W = engine.load_weights(engine.DEFAULT_UNIT)
graphs = [(1000,) + e for e in gmm_gpu.gmm_pairs(1000, range(nb), exact=True)]
eng = _lib.Engine(W)


def run(order, reps=5):
    eng.load_graphs([graphs[i] for i in order])
    eng.reset(); eng.rollout()
    best = 1e9
    for _ in range(reps):
        eng.reset()
        t0 = time.perf_counter(); out = eng.rollout(); dt = time.perf_counter() - t0
        best = min(best, eng.last_timing()[0])
    res = [None] * nb
    for k, i in enumerate(order):
        res[i] = out[k]
    return best, res


base_ms, base = run(list(range(nb)))
lens = np.array([len(o[0]) for o in base])
ne = np.array([len(g[1]) + len(g[2]) for g in graphs])
print("rollout lengths min/median/max %d/%d/%d; corr(len, edges) %.2f" % (
    lens.min(), np.median(lens), lens.max(), np.corrcoef(lens, ne)[0, 1]), flush=True)
print("seed order      %.2f ms -> %.0f removals/s" % (base_ms, lens.sum() / base_ms * 1e3), flush=True)
for name, order in [("edges desc", list(np.argsort(-ne, kind="stable"))),
                    ("length desc", list(np.argsort(-lens, kind="stable")))]:
    ms, res = run(order)
    same = all(np.array_equal(np.asarray(a[0]), np.asarray(b[0])) for a, b in zip(res, base))
    print("%-15s %.2f ms -> %.0f removals/s  same results %s" % (name, ms, lens.sum() / ms * 1e3, same), flush=True)
eng.close()
