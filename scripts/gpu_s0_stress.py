"""Repeat MvcEnv.s0 (reset) on golden graphs and report the max_rank distribution."""
import os, sys, collections
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdcommunity_amd import _lib, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
reps = int(os.environ.get("REPS", "40"))
for nm in sys.argv[1:] or ["er1000", "gmm1000_s0", "er300_dense"]:
    z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{nm}.npz"))
    n = int(z["n_nodes"])
    for team in (0, 2):
        eng.set_team_size(team)
        eng.load_graphs([(n, z["edges0"], z["edges1"])])
        c = collections.Counter(int(eng.reset()[0]) for _ in range(reps))
        print(nm, "team", team, "golden", int(z["max_rank"]), dict(c), flush=True)
    # batch of 4 copies (shared-mode phase A when disabled dedicated)
    eng.set_team_size(0)
    eng.load_graphs([(n, z["edges0"], z["edges1"])] * 20)
    c = collections.Counter(int(x) for _ in range(reps // 4) for x in eng.reset())
    print(nm, "batch20", dict(c), flush=True)
eng.close()
