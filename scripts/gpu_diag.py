"""Quick on-GPU parity/timing diagnostic against the golden fixtures."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdcommunity_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = dict(np.load(os.path.join(ROOT, "mdcommunity_amd/weights/unit_g0.5_iter100000.npz")))
MASK = -(2147483647 / 2)

def run(name, team=0):
    z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
    eng = _lib.Engine(_lib.pack_weights(W))
    if team: eng.set_team_size(team)
    n = int(z["n_nodes"])
    eng.load_graphs([(n, z["edges0"], z["edges1"])])
    mr = eng.reset()
    print(name, "max_rank", mr[0], "golden", int(z["max_rank"]), flush=True)
    # predict on s0 state
    q, am, nt, gap = eng.predict()
    gq = z["q_rows"][0]
    live = gq != MASK
    dq = np.abs(q[live].astype(np.float64) - gq[live])
    print(" predict: live match", np.array_equal(np.isfinite(q), live), "max|dq|", dq.max() if dq.size else 0,
          "exact frac", np.mean(q[live].astype(np.float64) == gq[live]), "argmax", am[0], "golden", int(z["seq"][0]), flush=True)
    # replay golden sequence
    ranks = []
    for a in z["seq"]:
        lm, term = eng.step(np.array([a]))
        ranks.append(int(lm[0]))
    print(" replay ranks match", ranks == z["ranks"].tolist(), "terminal", bool(term[0]), flush=True)
    if ranks != z["ranks"].tolist():
        bad = [i for i,(a,b) in enumerate(zip(ranks, z["ranks"])) if a!=b][:5]
        print("  first mismatches", bad, [ranks[i] for i in bad], [int(z["ranks"][i]) for i in bad])
    # full rollout
    eng.reset()
    t0 = time.time()
    out = eng.rollout()
    dt = time.time() - t0
    seq, rk = out[0]
    ms, nl = eng.last_timing()
    ok = seq.tolist() == z["seq"].tolist()
    score = 0.0
    for r in rk: score += r / (int(z["max_rank"]) * float(n))
    print(f" rollout: seq match {ok} len {len(seq)}/{len(z['seq'])} score {score} golden {float(z['score'])} "
          f"wall {dt*1e3:.2f} ms kernel {ms:.2f} ms launches {nl} -> {len(seq)/dt:.0f} rem/s", flush=True)
    if not ok:
        d = next((i for i,(a,b) in enumerate(zip(seq, z['seq'])) if a!=b), None)
        print("  first divergence at step", d, seq[d:d+3] if d is not None else None, z['seq'][d:d+3] if d is not None else None)
        tr = eng.trace(0)
        if d is not None:
            print("  trace at d: ntie", tr['n_tie'][d], 'gap', tr['gap'][d], 'golden gap', z['step_gap'][d], 'golden ntie', z['step_stats'][d][3])
    eng.close()

if __name__ == "__main__":
    names = sys.argv[1:] or ["er100", "gmm200_s7", "gmm1000_s0"]
    for nm in names:
        run(nm)
