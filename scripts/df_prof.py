"""Per-step phase profile of a dataflow-mode single-graph rollout (md_profile stamps: phase A
of the environment workgroup, tile 0's layer-0 workgroup, the graph-head workgroup)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine
W = engine.load_weights(engine.DEFAULT_UNIT)
name = sys.argv[1] if len(sys.argv) > 1 else "gmm1000_s0"
z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
e = _lib.Engine(W)
e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
e.reset(); e.rollout()
ks = []
for _ in range(10):
    e.reset(); e.rollout(); ks.append(e.last_timing()[0])
e.reset(); e.profile(512); e.rollout(); ms, _ = e.last_timing()
P = e.profile_read().astype(np.int64); e.profile(0)
S = len(P)
full = P[(P[:, 10] > 0) & (P[:, 0] > 0)]
nxt = np.append(P[1:, 0], 0)[(P[:, 10] > 0) & (P[:, 0] > 0)]
ok = nxt > 0
d = lambda a, b: (full[:, b] - full[:, a]) / 100.0
segs = [("phaseA", 0, 3), ("rec->tile", 3, 4), ("it1", 4, 5), ("it2 gather", 5, 23), ("it2 rest", 23, 6),
        ("it3 gather", 6, 29), ("it3 upd+norm", 29, 30), ("L1 recv", 30, 8), ("attn+Q", 8, 9)]
print(f"{name}: unprofiled kernel ms median {np.median(ks):.3f}; profiled {ms:.3f} ms, {len(full)} steps", flush=True)
print("  median us: " + "  ".join(f"{s}={np.median(d(a, b)):.1f}" for s, a, b in segs) +
      f"  tile end->next phaseA={np.median((nxt[ok] - full[ok, 9]) / 100.0):.1f}  step={np.median((nxt[ok] - full[ok, 0]) / 100.0):.1f}", flush=True)
print("  mean us:   " + "  ".join(f"{s}={np.mean(d(a, b)):.1f}" for s, a, b in segs) +
      f"  tile end->next phaseA={np.mean((nxt[ok] - full[ok, 9]) / 100.0):.1f}  step={np.mean((nxt[ok] - full[ok, 0]) / 100.0):.1f}", flush=True)
h = lambda a, b: np.median((full[:, b] - full[:, a]) / 100.0)
print("  head it3 from record: start %.1f graph_sum(S2) done %.1f vrow %.1f head %.1f published %.1f us" % (
    h(3, 49), h(3, 50), h(3, 51), h(3, 52), h(3, 53)), flush=True)
e.close()
