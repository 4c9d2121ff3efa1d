"""Single-graph rollouts with and without the dataflow mode (MD_DF): kernel ms per rollout
(median of 15) and the removal sequences / LMCC traces compared between the two modes."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine
W = engine.load_weights(engine.DEFAULT_UNIT)
names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["gmm1000_s0"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for name in names:
    z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
    g = (int(z["n_nodes"]), z["edges0"], z["edges1"])
    res = {}
    for df in ("0", "1", "0", "1"):
        os.environ["MD_DF"] = df
        e = _lib.Engine(W)
        e.load_graphs([g])
        e.reset()
        out = e.rollout()
        ts = []
        for _ in range(reps):
            e.reset()
            o2 = e.rollout()
            ts.append(e.last_timing()[0])
            assert list(o2[0][0]) == list(out[0][0]), "rollout differs between repeats"
        e.close()
        res.setdefault(df, []).append((float(np.median(ts)), float(np.min(ts)), out))
    seq0, seq1 = res["0"][0][2][0], res["1"][0][2][0]
    same = list(seq0[0]) == list(seq1[0]) and list(seq0[1]) == list(seq1[1])
    print("%s: %d removals; MD_DF=0 %s ms, MD_DF=1 %s ms (median / min per pass); identical rollouts: %s" % (
        name, len(seq0[0]), ["%.3f/%.3f" % r[:2] for r in res["0"]], ["%.3f/%.3f" % r[:2] for r in res["1"]], same),
        flush=True)
