"""Where the mutual-LMCC fixed point's time goes over a single-graph rollout: phase A runs every
fixed point itself (MD_SPEC=0), md_profile's round accounting (slots 16-22, 56 of each step)
summed over the steps.  python scripts/fp_prof.py [golden name] (MD_FP_SHORTCUT honoured)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MD_SPEC"] = "0"
from mdcommunity_amd import _lib, engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "gmm1000_s0"
z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
for _ in range(3):
    e.reset()
    e.rollout()
e.reset()
e.profile(512)
e.rollout()
ms, _ = e.last_timing()
P = e.profile_read().astype(np.int64)
e.profile(0)
e.close()
P = P[P[:, 21] > 0]  # steps whose phase A ran a fixed point
tot = lambda c: P[:, c].sum() / 100.0
print(f"{name} MD_FP_SHORTCUT={os.environ.get('MD_FP_SHORTCUT', '1')}: kernel {ms:.3f} ms (MD_SPEC=0), {len(P)} fixed points, "
      f"{P[:, 16].sum()} rounds; us total: init {tot(56):.0f} unite {tot(17):.0f} label {tot(18):.0f} prune+check {tot(19):.0f} "
      f"count {tot(20):.0f} cover {tot(22):.0f}; per fixed point {(tot(56) + tot(17) + tot(18) + tot(19) + tot(20)) / len(P):.1f} us",
      flush=True)
# per fixed point (first 12 and the slowest 5): rounds and the round accounting in us
rows = lambda idx: "\n".join(f"  fp {i:3d}: rounds {P[i, 16]:2d}  init {P[i, 56] / 100:.1f}  unite {P[i, 17] / 100:.1f}  label {P[i, 18] / 100:.1f}  "
                             f"prune+check {P[i, 19] / 100:.1f}  count {P[i, 20] / 100:.1f}" for i in idx)
print(rows(range(min(12, len(P)))), flush=True)
cost = P[:, 56] + P[:, 17] + P[:, 18] + P[:, 19] + P[:, 20]
print("  slowest:\n" + rows(np.argsort(-cost)[:5]), flush=True)
