"""On-GPU phase profile of the rollout kernel (workgroup-0 wall-clock stamps)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdcommunity_amd import _lib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = _lib.pack_weights(dict(np.load(os.path.join(ROOT, "mdcommunity_amd/weights/unit_g0.5_iter100000.npz"))))
NAMES = ["A:mcc", "A:feat", "A:end", "barA", "p1", "bar1", "p2", "bar2", "p3", "bar3"]

def prof(name, team):
    if name == "real":  # the testReal-sized synthetic multiplex (mdcommunity_amd.synth, N = 18000)
        from mdcommunity_amd import synth
        layers = synth.real_like_layers(18000, 0)
        n = 18000
        es = []
        for lay in layers:
            seen, order = set(), []
            for u, v in lay:
                k = (min(u, v), max(u, v))
                if u != v and k not in seen:
                    seen.add(k)
                    order.append(k)
            es.append(np.array(sorted(order), np.int32))
        z = {"edges0": es[0], "edges1": es[1], "seq": np.zeros(1)}
    else:
        z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
        n = int(z["n_nodes"])
    eng = _lib.Engine(W)
    eng.set_team_size(team)
    eng.load_graphs([(n, z["edges0"], z["edges1"])])
    eng.reset()
    eng.rollout()  # warm
    kms = []
    for _ in range(15):  # unprofiled device time per rollout
        eng.reset()
        eng.rollout()
        kms.append(eng.last_timing()[0])
    print(f"{name}: unprofiled rollout kernel ms: median {np.median(kms):.3f} min {np.min(kms):.3f} "
          f"-> {np.median(kms) / len(z['seq']) * 1000:.1f} us per removal", flush=True)
    tr_n = eng.trace(0)["n_live"]
    eng.reset()
    eng.profile(512)
    t0 = time.time(); out = eng.rollout(); dt = time.time() - t0
    ms, nl = eng.last_timing()
    P = eng.profile_read().astype(np.int64)
    eng.profile(0)
    # slots: 0 startA,1 after mcc,2 after feat,3 endA,4 afterbarA,11 p1 tiles start,5 end p1,6 after bar1,12,7,8,13,9,10
    full = P[(P[:, 10] > 0)]
    d = lambda a, b: np.median((full[:, b] - full[:, a])) * 10 / 1000.0  # us
    seg = [("A:stage", 0, 1), ("A:apply+mcc", 1, 2), ("A:deg", 2, 32), ("A:live", 32, 34), ("A:wb", 34, 14), ("A:h0", 14, 15), ("A:wreload", 15, 3), ("barA", 3, 4), ("pref", 4, 11), ("p1", 11, 5), ("bar1", 5, 6), ("p2", 12, 7),
           ("bar2", 7, 8), ("p3", 13, 9), ("bar3", 9, 10)]
    tot = np.median(full[:, 10] - full[:, 0]) * 10 / 1000.0
    print(f"{name} team={team} variant={os.environ.get('MD_VARIANT', '0')} env_mode={os.environ.get('MD_ENV_MODE', '1')}: removals {len(out[0][0])} wall {dt*1e3:.2f} ms kernel {ms:.2f} ms launches {nl}; "
          f"steps profiled {len(full)} median step {tot:.1f} us", flush=True)
    print("   " + "  ".join(f"{s}={d(a,b):.1f}" for s, a, b in seg), flush=True)
    dm = lambda a, b: np.mean((full[:, b] - full[:, a])) * 10 / 1000.0
    print("   mean: " + "  ".join(f"{s}={dm(a,b):.1f}" for s, a, b in seg), flush=True)
    stp = (full[:, 10] - full[:, 0]) / 100.0
    print("   sum of step times %.3f ms (kernel %.3f ms); first step %.1f us; top-5 steps %s us at %s" % (
        stp.sum() / 1000, ms, stp[0], np.round(np.sort(stp)[-5:], 1).tolist(), np.argsort(stp)[-5:].tolist()), flush=True)
    stp_ = (full[:, 10] - full[:, 0]) / 100.0
    show = sorted(set(list(range(min(4, len(full)))) + np.argsort(stp_)[-8:].tolist()))
    for t in show:
        acc_ = full[t, 16:23]
        print("   step %2d (n_live %d): %s | rounds %d unite %.1f label %.1f prune %.1f" % (t, tr_n[t] if t < len(tr_n) else -1, "  ".join(
            f"{s}={(full[t, b] - full[t, a]) / 100:.1f}" for s, a, b in seg), acc_[0], acc_[1] / 100, acc_[2] / 100, acc_[3] / 100), flush=True)
    tt = lambda a, b: np.median((full[:, b].astype(np.int64) - full[:, a].astype(np.int64))) / 100.0
    print("   tile wg: p1 gather %.1f upd %.1f end %.1f | p2 gather %.1f upd %.1f end %.1f | p3 gather %.1f upd %.1f attn %.1f us" % (
        tt(11, 23), tt(23, 24), tt(24, 25), tt(12, 26), tt(26, 27), tt(27, 28), tt(13, 29), tt(29, 30), tt(30, 31)), flush=True)
    print("   head it3 (from barrier 2 exit): start %.1f gv %.1f graph_sum %.1f vrow %.1f graph_head %.1f publish %.1f -> done at %.1f us" % (
        tt(8, 48), tt(48, 49), tt(49, 50), tt(50, 51), tt(51, 52), tt(52, 53), tt(8, 53)), flush=True)
    print("   it1 gather detail: rows %.1f | lists: rowptr %.1f prefix %.1f flags+scan %.1f pass2 %.1f offsets %.1f | gather %.1f us" % (
        tt(11, 54), tt(54, 60), tt(60, 61), tt(61, 62), tt(62, 63), tt(63, 55), tt(55, 23)), flush=True)
    print("   tile it1: update %.1f normalize %.1f sums+stores %.1f | attn: tanh %.1f dots+gates %.1f mix %.1f norm %.1f head-wait %.1f e-chain %.1f hidden+Q %.1f argmax %.1f us" % (
        tt(23, 36), tt(36, 37), tt(37, 24), tt(29, 38), tt(38, 33), tt(33, 35), tt(35, 39), tt(39, 40), tt(40, 41), tt(41, 42), tt(42, 31)), flush=True)
    print("   slowest tile end (from barrier exit): it1 %.1f it2 %.1f it3 %.1f us" % (tt(11, 43), tt(12, 44), tt(13, 45)), flush=True)
    print("   it2: latest tile start %.1f us after WG0 exit, longest gather %.1f us" % (tt(12, 47), np.median(full[:, 46].astype(np.float64)) / 100), flush=True)
    ex = full[:, 56:60].astype(np.float64)
    print("   env extra: init %.1f us  alive edges/step (MD_VARIANT=8) %.0f" % (np.median(ex[:, 0]) / 100, np.median(ex[:, 2])), flush=True)
    if np.any(ex[:, 2] > 0):
        acc_ = full[:, 16:23].astype(np.float64)
        rate = acc_[:, 1] / 100 / np.maximum(ex[:, 2], 1) * 1000
        q = np.percentile(np.arange(len(full)), [0, 25, 50, 75, 100]).astype(int)
        print("   unite us per 1000 edge-rounds at steps %s: %s; edges/step %s; mean forest depth %s" % (
            q.tolist(), np.round(rate[q], 2).tolist(), ex[q, 2].astype(int).tolist(),
            np.round(ex[q, 1] / np.maximum(acc_[q, 0], 1) / 2000, 2).tolist()), flush=True)
    acc = full[:, 16:23].astype(np.float64)
    calls = np.maximum(acc[:, 5], 1)
    print("   env per step: rounds/call %.2f  cover %.1f  unite %.1f  label %.1f  prune %.1f  count %.1f us" % (
        np.mean(acc[:, 0] / calls), np.median(acc[:, 6]) / 100, np.median(acc[:, 1]) / 100,
        np.median(acc[:, 2]) / 100, np.median(acc[:, 3]) / 100, np.median(acc[:, 4]) / 100), flush=True)
    eng.close()

def batch(nb, team):
    gs = []
    for name in ["gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000"]:
        z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
        gs.append((int(z["n_nodes"]), z["edges0"], z["edges1"], len(z["seq"])))
    eng = _lib.Engine(W)
    eng.set_team_size(team)
    sel = [gs[i % 4] for i in range(nb)]
    eng.load_graphs([g[:3] for g in sel])
    eng.reset(); eng.rollout(); eng.reset()
    t0 = time.time(); out = eng.rollout(); dt = time.time() - t0
    ms, nl = eng.last_timing()
    rem = sum(len(o[0]) for o in out)
    print(f"batch {nb} team={team}: removals {rem} wall {dt*1e3:.1f} ms kernel {ms:.1f} ms launches {nl} -> {rem/dt:.0f} rem/s", flush=True)
    eng.close()

if __name__ == "__main__":
    for team in [int(x) for x in sys.argv[1].split(",")]:
        prof(os.environ.get("MD_PROF_GRAPH", "gmm1000_s0"), team)
    if len(sys.argv) > 2:
        for nb in [int(x) for x in sys.argv[2].split(",")]:
            batch(nb, 0)
