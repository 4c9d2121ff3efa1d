"""Where a prediction of the testReal-sized rollout goes (N = 18 000 synthetic multiplex,
mdcommunity_amd.synth, the bench's real_scale object): workgroup 0's phase stamps of the
lock-step kernel (md_profile) split each step into the grid-wide environment step (team_env_step,
stamps 0 -> 3), barrier A (3 -> 4) and the three message-passing iterations with their barriers
(4 -> 10), plus the team step's own pieces (slots 80-87, scripts/team_prof.py) and the union
pass's per-thread counts (slots 88-95: parent loads and compare-and-swaps, failed ones, the
longest union, the slowest workgroup's union and label work).
Usage: python scripts/real_prof.py [degree|unit] [n]"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, agent, engine, graph as mgraph, synth  # noqa: E402

cost = sys.argv[1] if len(sys.argv) > 1 else "degree"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 18000
with tempfile.TemporaryDirectory() as td:
    path = os.path.join(td, "real_like_multiplex.edges")
    synth.write_real_like(path, n, seed=0)
    a = agent.MultiDismantler.__new__(agent.MultiDismantler)
    _, gl = agent.MultiDismantler.read_multiplex(a, path, n)
e0, e1 = np.asarray(gl[0], np.int32), np.asarray(gl[1], np.int32)
g = mgraph.Graph_test.from_edges(n, e0, e1)
if cost == "degree":
    mgraph.ensure_degree_weights(g)
    eng = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
    eng.load_graphs([(n, e0, e1)], node_w=mgraph.node_weight_array([g]))
    step = 1
else:
    eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT_REAL))
    eng.load_graphs([(n, e0, e1)])
    step = max(1, int(0.01 * n))
eng.reset()
eng.rollout(step=step)  # warm
kms = []
for _ in range(3):
    eng.reset()
    seq, _ = eng.rollout(step=step)[0]
    kms.append(eng.last_timing()[0])
npred = len(eng.trace(0)["n_live"])
print(f"{cost} N={n}: {len(seq)} removals, {npred} predictions, rollout kernel median {np.median(kms):.2f} ms "
      f"= {np.median(kms) / max(1, npred) * 1e3:.0f} us per prediction", flush=True)
eng.reset()
eng.profile(4096)
eng.rollout(step=step)
ms = eng.last_timing()[0]
P = eng.profile_read().astype(np.int64)
eng.profile(0)
R = P[P[:, 10] > 0]
us = lambda a, b: (R[:, b] - R[:, a]) / 100.0
parts = [("env", 0, 3), ("barA", 3, 4), ("it1", 11, 5), ("bar1", 5, 6), ("it2", 12, 7), ("bar2", 7, 8),
         ("it3", 13, 9), ("bar3", 9, 10), ("step", 0, 10)]
print(f"profiled rollout {ms:.2f} ms, {len(R)} steps with every stamp", flush=True)
print("  median us: " + "  ".join(f"{k} {np.median(us(a, b)):.1f}" for k, a, b in parts), flush=True)
print("  mean us:   " + "  ".join(f"{k} {np.mean(us(a, b)):.1f}" for k, a, b in parts), flush=True)
print("  sums ms:   " + "  ".join(f"{k} {us(a, b).sum() / 1e3:.2f}" for k, a, b in parts), flush=True)
T = R[R[:, 87] > 0]
if len(T):
    rd = np.maximum(T[:, 80], 1)
    nm = ["union", "label+reduce", "prune+reduce", "count", "features", "inits"]
    print("  team step: rounds median %.0f mean %.2f; median us %s" % (
        np.median(T[:, 80]), T[:, 80].mean(), "  ".join("%s %.1f" % (k, np.median(T[:, 81 + i]) / 100) for i, k in enumerate(nm))),
          flush=True)
    print("  union pass per round: workgroup 0's own work %.1f us, slowest workgroup's %.1f us (median over steps)" % (
        np.median(T[:, 88] / rd) / 100, np.median(T[:, 89]) / 100), flush=True)
    un = np.maximum(T[:, 92], 1)
    print("  unions: %.0f per step, parent loads + CASes per union %.2f (mean), most by one thread %d (median "
          "over steps; max %d), failed CASes per union %.4f, longest union %.2f us (median; max %.2f); slowest "
          "workgroup's label work %.1f us" % (
              np.median(T[:, 92]), np.median(T[:, 91] / un), np.median(T[:, 90]), T[:, 90].max(),
              np.median(T[:, 94] / un), np.median(T[:, 93]) / 100, T[:, 93].max() / 100, np.median(T[:, 95]) / 100),
          flush=True)
    print("  team step per round us: union %.1f label %.1f" % (
        np.median(T[:, 81] / rd) / 100, np.median(T[:, 82] / rd) / 100), flush=True)
eng.close()
