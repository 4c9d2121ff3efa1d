"""Single-graph rollouts under settings of one environment switch (AB_VAR, default MD_DF, values
AB_MODES / DF_MODES, default 0,1): kernel ms per rollout (median of 15) and the removal
sequences / LMCC traces compared between the settings."""
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
    var = os.environ.get("AB_VAR", "MD_DF")
    modes = os.environ.get("AB_MODES", os.environ.get("DF_MODES", "0,1")).split(",")
    for df in modes + modes:
        os.environ[var] = df
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
    seq0 = res[modes[0]][0][2][0]
    same = all(list(res[m][0][2][0][0]) == list(seq0[0]) and list(res[m][0][2][0][1]) == list(seq0[1]) for m in modes)
    print("%s: %d removals; " % (name, len(seq0[0])) + "; ".join("%s=%s %s ms" % (var, m, ["%.3f/%.3f" % r[:2] for r in res[m]]) for m in modes) +
          " (median / min per pass); identical rollouts: %s" % same, flush=True)
