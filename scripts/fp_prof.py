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
