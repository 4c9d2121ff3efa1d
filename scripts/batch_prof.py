"""Per-step phase profile of a batched rollout launch (shared mode): workgroup-0 wall-clock
stamps per removal step, next to the active graphs and live-node tiles of that step."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
W = engine.load_weights(engine.DEFAULT_UNIT)
graphs = [(1000,) + gmm.gmm_pair(1000, seed=s) for s in range(nb)]
eng = _lib.Engine(W)
eng.load_graphs(graphs)
eng.reset(); eng.rollout()
eng.reset()
t0 = time.time(); out = eng.rollout(); dt = time.time() - t0
ms, nl = eng.last_timing()
lens = np.array([len(o[0]) for o in out])
print(f"batch {nb}: removals {lens.sum()} kernel {ms:.2f} ms wall {dt*1e3:.1f} ms -> {lens.sum()/dt:.0f} rem/s; "
      f"rollout length min/median/max {lens.min()}/{int(np.median(lens))}/{lens.max()}", flush=True)
# per-step work from the device traces
S = lens.max() + 1
act = np.zeros(S, int); tiles = np.zeros(S, int); nodes = np.zeros(S, int)
for g in range(nb):
    tr = eng.trace(g)
    for t, n_t in enumerate(tr["n_live"]):
        act[t] += 1; tiles[t] += (int(n_t) + 15) // 16; nodes[t] += int(n_t)
eng.reset()
eng.profile(512)
eng.rollout()
ms2, _ = eng.last_timing()
P = eng.profile_read().astype(np.int64)
eng.profile(0)
if len(P) and P[0, 0] == 1 and P[0, 9] > 0:
    # queue mode: per item kind total device time (summed over workgroups) and counts
    names = {1: "ENV", 3: "VN 1", 4: "VN 2", 5: "TILE it1", 6: "TILE it2", 7: "TILE it3"}
    cnt = {1: P[0, 9], 3: P[0, 11], 5: P[0, 10]}
    tot = P[0, 16] + P[0, 17] + sum(P[0, k] for k in names)
    print("queue mode, %.1f WG-ms in total (%d workgroups x %.2f ms)" % (tot / 1e5, 256, ms2 / 1.0))
    for k, nm in names.items():
        print("  %-9s %9.1f WG-ms" % (nm, P[0, k] / 1e5))
    print("  items: ENV %d VN %d TILE %d; waiting for items %.1f WG-ms; weight reloads %.1f WG-ms" % (
        P[0, 9], P[0, 11], P[0, 10], P[0, 16] / 1e5, P[0, 17] / 1e5))
    npop = P[0, 9] + P[0, 10] + P[0, 11]
    print("  pops with the slot filled at the early read: %d of ~%d; mean backlog beyond the held ticket %.1f items" % (
        P[0, 18], npop, P[0, 19] / max(1, npop)))
    if os.environ.get("MD_VARIANT", "0") != "0" and int(os.environ["MD_VARIANT"]) & 8:
        names_t = ["header", "nb lists", "gather", "update", "normalize", "sums+stores", "attn+Q"]
        for it in range(3):
            row = P[0, 20 + 8 * it: 27 + 8 * it] / 1e5
            cnt = max(1, {0: 1, 1: 1, 2: 1}[it])
            print("  TILE it%d pieces (WG-ms): " % (it + 1) + "  ".join("%s %.1f" % (nm, v) for nm, v in zip(names_t, row)))
        env_n = ["stage", "fixed point", "features", "write-back", "h0 table"]
        print("  ENV pieces (WG-ms): " + "  ".join("%s %.1f" % (nm, v) for nm, v in zip(env_n, P[0, 80:85] / 1e5)) +
              " | phase A total %.1f  neighbour lists %.1f" % (P[0, 85] / 1e5, P[0, 86] / 1e5))
        if P[0, 62] > 0:
            print("  paired gather: own loads + first batch in flight %.1f WG-ms, batch loop %.1f WG-ms; %.2f batches and %.0f list entries per gather" % (
                P[0, 60] / 1e5, P[0, 61] / 1e5, P[0, 62] / max(1, P[0, 10] * 0.5), P[0, 63] / max(1, P[0, 10] * 0.5)))
        if P[0, 64] > 0:
            print("  paired gather batches, iterations 2-3 (every thread's loads in, then a barrier): waiting for the loads %.1f WG-ms, staging stores + adds + barriers %.1f WG-ms" % (
                P[0, 64] / 1e5, P[0, 65] / 1e5))
        if P[0, 44] > 0:
            wn = ["phase A", "park check", "lists", "push", "weight reload"]
            print("  wave ENV pieces (WG-ms): " + "  ".join("%s %.1f" % (nm, v) for nm, v in zip(wn, P[0, 44:49] / 1e5)))
        if P[0, 50] > 0:
            ln = ["live positions", "prefixes", "entries + alive counts", "scan + list stores", "headers"]
            print("  ENV list builder pieces (WG-ms): " + "  ".join("%s %.1f" % (nm, v) for nm, v in zip(ln, P[0, 50:55] / 1e5)))
        att_n = ["tanh GEMM", "dots+gates", "mix+norm", "head", "e-chain", "hidden+Q", "arg-max+stores"]
        print("  attention pieces (WG-ms): " + "  ".join("%s %.1f" % (nm, v) for nm, v in zip(att_n, P[0, 88:95] / 1e5)))
        sys.exit(0)
    wb = P[0, 20:64] / 1e5
    nb_ = int(np.max(np.nonzero(wb)[0])) + 1 if np.any(wb) else 0
    print("  idle workgroups per 1.31 ms of the launch: " + " ".join("%.0f" % (w / 1.31) for w in wb[:nb_]))
    sys.exit(0)
full = P[P[:, 10] > 0]
d = lambda a, b: (full[:, b] - full[:, a]) / 100.0
A, bA, i1, i2, i3 = d(0, 3), d(3, 4), d(4, 6), d(6, 8), d(8, 10)
tot = d(0, 10)
print(f"profiled kernel {ms2:.2f} ms, steps {len(full)}; sum of step times {tot.sum()/1000:.2f} ms", flush=True)
print("phase totals ms: A %.2f barA %.2f it1 %.2f it2 %.2f it3 %.2f" % (A.sum()/1e3, bA.sum()/1e3, i1.sum()/1e3, i2.sum()/1e3, i3.sum()/1e3))
# (profiled steps include the steps where every running graph waited for a host answer, so
# the work columns are exact only up to the first tie)
for t in list(range(0, min(len(full), 12))) + list(range(12, len(full), max(1, len(full)//20))):
    wk = (act[t], tiles[t], nodes[t]) if t < S else (0, 0, 0)
    print(f"step {t:4d}: active {wk[0]:4d} tiles {wk[1]:6d} nodes {wk[2]:7d} | A {A[t]:7.1f} barA {bA[t]:5.1f} it1 {i1[t]:7.1f} it2 {i2[t]:7.1f} it3 {i3[t]:7.1f} us", flush=True)
eng.close()
