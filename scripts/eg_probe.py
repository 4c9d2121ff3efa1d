"""K2 end-game cost of a single-graph rollout (gmm1000_s0): the kernel time of plain rollouts
and the phase-A stamps of the last steps (slot 0: phase A start, 1: the action loop's start,
2: its end, 3: phase A end; md_profile rows, 100 MHz clock), with the end-game answer applied
in one pass (MD_EG_APPLY=1) and action by action (0)."""
import os
import sys

import numpy as np

ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine  # noqa: E402

z = np.load(os.path.join(ROOT, "tests/golden/rollout_gmm1000_s0.npz"))
graph = (int(z["n_nodes"]), z["edges0"], z["edges1"])
for apply in ("1", "0"):
    os.environ["MD_EG_APPLY"] = apply
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    e.load_graphs([graph])
    ts = []
    for _ in range(21):
        e.reset()
        seq, _ = e.rollout()[0]
        ts.append(e.last_timing()[0])
    e.reset()
    e.profile(512)
    e.rollout()
    P = e.profile_read().astype(np.int64)
    e.profile(0)
    rows = [i for i in range(len(P)) if P[i, 0] > 0]
    t0 = P[rows[0], 0]
    print(f"MD_EG_APPLY={apply}: removals {len(seq)}, kernel ms median {np.median(ts[1:]):.4f} min {min(ts[1:]):.4f}")
    for i in rows[-3:]:
        print("  row", i, [(k, round((P[i, k] - t0) / 100.0, 1)) for k in range(0, 4) if P[i, k] > 0])
    e.close()
