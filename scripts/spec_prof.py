#!/usr/bin/env python3
"""Timeline of the speculative environment steps (md_profile slots 64-72) of single-graph
rollouts: request -> speculative workgroup 0 (seen, candidate, staged, done) and the next
phase A's check (start, hit slot, end, the hit result's done time), in us after the request.
Usage: python scripts/spec_prof.py [fixture] (MD_SPEC sets the workgroup count)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "gmm1000_s0"
z = np.load(os.path.join(ROOT, "tests", "golden", f"rollout_{name}.npz"))
n = int(z["n_nodes"])
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
eng.load_graphs([(n, z["edges0"], z["edges1"])])
kms = []
for _ in range(10):
    eng.reset()
    eng.rollout()
    kms.append(eng.last_timing()[0])
hits, rem = eng.spec_stats(0)
print(f"{name} MD_SPEC={os.environ.get('MD_SPEC', '16')}: kernel ms median {np.median(kms):.3f} "
      f"({np.median(kms) / rem * 1e3:.1f} us per removal); spec hits {hits} of {rem} removals", flush=True)
eng.reset()
eng.profile(512)
eng.rollout()
P = eng.profile_read().astype(np.int64)
eng.profile(0)
rows = P[P[:, 64] > 0]
us = lambda a, b: (rows[:, b] - rows[:, a]) / 100.0
have = rows[:, 68] > 0
chk = rows[:, 69] > 0
hit = rows[:, 70] > 0
print(f"requests {len(rows)}; wg0 done {have.sum()}; checks {chk.sum()}; hits {hit.sum()}")
med = lambda x: float(np.median(x)) if len(x) else float("nan")
print("wg0 (us after request): seen %.1f  loaded %.1f  candidate %.1f  taken %.1f  done %.1f  features %.1f" % (
    med(us(64, 65)[have]), med(us(64, 73)[have]), med(us(64, 66)[have]), med(us(64, 67)[have]), med(us(64, 68)[have]),
    med(us(64, 74)[have])))
print("next phase A (us after request): check start %.1f  check end %.1f (wait %.1f, mean %.1f); hit result done %.1f" % (
    med(us(64, 69)[chk]), med(us(64, 71)[chk]), med(us(69, 71)[chk]), float(np.mean(us(69, 71)[chk])), med(us(64, 72)[hit])))
print("features copied in %d of %d profiled steps" % (int((P[:, 75] > 0).sum()), len(P)))
print("hit slots (rank + 1):", np.bincount(rows[:, 70][chk].astype(int), minlength=17).tolist())
late = us(69, 71)[chk]
print("waits > 5 us: %d; largest %s" % ((late > 5).sum(), np.round(np.sort(late)[-8:], 1).tolist()))
pre = P[:, 78]
pre = pre[pre > 0] - 1
if len(pre):
    print("iteration-1 prebuild per step (first tile workgroup): whole iteration used %d, lists used %d, built but not "
          "confirmed %d, not built %d of %d steps" % (int(np.sum(pre % 10 == 3)), int(np.sum((pre % 10 > 0) & (pre % 10 < 3))),
                                                  int(np.sum((pre // 10 > 0) & (pre % 10 == 0))), int(np.sum(pre // 10 == 0)),
                                                  len(pre)), flush=True)
