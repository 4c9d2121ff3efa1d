"""Piece profile of the batched-prefix environment step (md_env.h team_prefix_step) on the
testReal-sized synthetic multiplex (N = 18000), unit cost, stepRatio 0.01 (180 picks per
prediction): per prediction the prefixes, the most fixed-point rounds of any prefix, the slowest
prefix's fixed point, and the last (largest) prefix's pieces (md_profile slots 80-93)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 18000
step = max(int(0.01 * n), 1)
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
eng.rollout(step=step)
eng.reset()
eng.profile(4096)
seq, _ = eng.rollout(step=step)[0]
ms, _ = eng.last_timing()
P = eng.profile_read().astype(np.int64)
eng.profile(0)
R = P[:2048][P[:2048, 92] > 0]
print(f"N={n}, step {step}: {len(seq)} removals, rollout kernel {ms:.2f} ms; {len(R)} prefix batches", flush=True)
for r in R:
    us = lambda k: r[k] / 100.0
    print(f"  prefixes {r[92]} applied {r[93]}: most rounds {r[80]}; list+validation {us(81):.1f} us, slowest prefix "
          f"{us(82):.1f} us, death steps {us(83):.1f} us; last prefix ({r[91]} rounds): init {us(84):.1f} union "
          f"{us(86):.1f} labels {us(88):.1f} prune {us(89):.1f} lmcc+stores {us(90):.1f} us; step total {us(87):.1f} us")
if os.environ.get("MD_PROF_ALL") == "1" and len(P) > 2048:
    flat = np.zeros(24 * 96, np.int64)
    blk = P[2048:2048 + 24].reshape(-1)
    flat[:len(blk)] = blk
    rounds, ticks = flat[:1024], flat[1024:2048] / 100.0
    k = int(np.count_nonzero(rounds))
    print(f"  last batch, per prefix j=1..{k}: rounds " + " ".join(str(int(x)) for x in rounds[:k]))
    print("  fixed-point us: " + " ".join("%.0f" % x for x in ticks[:k]))
