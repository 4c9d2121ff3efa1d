"""Piece profile of the grid-wide environment step (team_env_step) on the testReal-sized
synthetic multiplex (N = 18000): per step the fixed-point rounds and the device time of each
pass kind (md_profile slots 80-87 of workgroup 0), medians over the profiled steps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 18000
es = []
for lay in synth.real_like_layers(n, 0):
    seen, order = set(), []
    for u, v in lay:
        k = (min(u, v), max(u, v))
        if u != v and k not in seen:
            seen.add(k)
            order.append(k)
    es.append(np.array(order, np.int32))
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT_REAL))
eng.load_graphs([(n, es[0], es[1])])
eng.reset()
eng.rollout()
eng.reset()
eng.profile(4096)
seq, _ = eng.rollout()[0]
ms, _ = eng.last_timing()
P = eng.profile_read().astype(np.int64)
eng.profile(0)
R = P[P[:, 87] > 0]
us = lambda k: R[:, k] / 100.0
print(f"N={n}: {len(seq)} removals, rollout kernel {ms:.1f} ms ({ms / len(seq) * 1e3:.0f} us per removal); "
      f"{len(R)} team steps profiled", flush=True)
names = ["union", "label+reduce", "prune+reduce", "count", "features", "inits", "step total"]
print("  rounds per step: median %.0f mean %.1f max %d" % (np.median(R[:, 80]), R[:, 80].mean(), R[:, 80].max()))
print("  median us: " + "  ".join("%s %.1f" % (nm, np.median(us(81 + i))) for i, nm in enumerate(names)))
print("  mean us:   " + "  ".join("%s %.1f" % (nm, np.mean(us(81 + i))) for i, nm in enumerate(names)))
rd = np.maximum(R[:, 80], 1)
print("  per round us: union %.1f label %.1f prune %.1f" % (np.median(us(81) / rd), np.median(us(82) / rd),
                                                          np.median(us(83) / np.maximum(rd - 1, 1))))
tot_team = R[:, 87].sum() / 1e5
print("  team steps %.1f ms of the %.1f ms rollout kernel (the rest: decisions, barriers, forward passes)" % (tot_team, ms))
print("  union pass: workgroup 0's own work %.1f us per round, slowest workgroup %.1f us (one round's max, median over steps)" % (
    np.median(R[:, 88] / rd) / 100, np.median(R[:, 89]) / 100))
