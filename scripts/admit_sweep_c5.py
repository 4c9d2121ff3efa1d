"""Admission-limit sweep of the one-launch C5 batch (4096 GMM N=1000 graphs, seeds 0..4095,
device generator exact mode): kernel time per batch rollout for each MD_VARIANT admission
value (bits 16+), graphs generated once.
  python scripts/admit_sweep_c5.py [graphs] [admits comma-separated] [reps]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm_gpu
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
admits = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,96,160,256,384").split(",")]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
W = engine.load_weights(engine.DEFAULT_UNIT)
t0 = time.time()
graphs = [(1000,) + tuple(e) for e in gmm_gpu.gmm_pairs(1000, range(nb), exact=True)]
print(f"generated {nb} graphs in {time.time() - t0:.1f} s", flush=True)
for a in admits:
    os.environ["MD_VARIANT"] = str(a << 16)
    eng = _lib.Engine(W)
    eng.load_graphs(graphs)
    eng.reset(); out = eng.rollout()
    rem = sum(len(o[0]) for o in out)
    ts, ws = [], []
    for _ in range(reps):
        tw = time.perf_counter()
        eng.reset(); eng.rollout()
        ws.append((time.perf_counter() - tw) * 1e3)
        ts.append(eng.last_timing())
    eng.close()
    best = min(ts)
    print(f"admit {a or 'default'}: removals {rem} kernel ms {best[0]:.1f} ({best[1]} launches) -> "
          f"{rem / best[0] * 1e3:.0f} removals/s; wall ms {min(ws):.1f} -> {rem / min(ws) * 1e3:.0f}", flush=True)
