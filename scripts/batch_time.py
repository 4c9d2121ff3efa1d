"""Best-of-K kernel time of one queue-mode launch over the C3 batch (256 GMM N=1000 graphs,
seeds 0..255, device generator exact mode); optional second column with another env setting:
  python scripts/batch_time.py [graphs] [reps] [ENV=VAL,...]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
if len(sys.argv) > 3:
    for kv in sys.argv[3].split(","):
        k, v = kv.split("=")
        os.environ[k] = v
from mdcommunity_amd import _lib, engine, gmm_gpu
W = engine.load_weights(engine.DEFAULT_UNIT)
graphs = [(1000,) + e for e in gmm_gpu.gmm_pairs(1000, range(nb), exact=True)]
eng = _lib.Engine(W)
eng.load_graphs(graphs)
eng.reset(); out = eng.rollout()
rem = sum(len(o[0]) for o in out)
lmax = max(len(o[0]) for o in out)
if os.environ.get("MD_LENS"):
    L = np.sort([len(o[0]) for o in out])[::-1]
    print("rollout lengths, longest first:", " ".join(str(x) for x in L[:24]), "... graphs longer than 40/60/80:",
          (L > 40).sum(), (L > 60).sum(), (L > 80).sum(), flush=True)
ts, ws = [], []
for _ in range(reps):
    t0 = time.perf_counter()
    eng.reset(); eng.rollout()
    ws.append((time.perf_counter() - t0) * 1e3)
    ts.append(eng.last_timing()[0])
ts.sort(); ws.sort()
print("batch %d (%s): removals %d, kernel ms best %.2f median %.2f -> %.0f removals/s; wall (reset + rollout) median %.2f ms -> %.0f removals/s" % (
    nb, sys.argv[3] if len(sys.argv) > 3 else "default", rem, ts[0], ts[len(ts) // 2], rem / ts[len(ts) // 2] * 1e3,
    ws[len(ws) // 2], rem / ws[len(ws) // 2] * 1e3), flush=True)
print("  longest rollout %d removals: %.1f us of kernel per step of it" % (lmax, ts[len(ts) // 2] * 1e3 / lmax), flush=True)
if os.environ.get("MD_HITS"):  # speculative environment steps taken, over the batch (last rollout)
    hs = [eng.spec_stats(g) for g in range(nb)]
    print("  speculative steps taken: %d of %d removals" % (sum(h for h, _ in hs), sum(r for _, r in hs)), flush=True)
eng.close()
