"""Piece profile of MvcEnv.s0 (md_reset: the initial mutual-LMCC prune) on the headline graph:
phase-A stamps and the fixed point's round accounting (md_profile slots 0-22 of step 0)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm  # noqa: E402

e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
e.load_graphs([(1000,) + gmm.gmm_pair(1000, seed=0)])
for _ in range(3):
    e.reset()
e.profile(4)
e.reset()
ms, _ = e.last_timing()
P = e.profile_read().astype(np.int64)
e.profile(0)
r = P[0]
t = lambda a, b: (r[b] - r[a]) / 100.0
print(f"s0 kernel {ms * 1e3:.1f} us: stage {t(0, 1):.1f} fixed point {t(1, 2):.1f} features {t(2, 34):.1f} "
      f"write-back {t(34, 14):.1f} h0 {t(14, 15):.1f} us | rounds {r[16]} unite {r[17] / 100:.1f} label {r[18] / 100:.1f} "
      f"prune {r[19] / 100:.1f} count {r[20] / 100:.1f} us", flush=True)
