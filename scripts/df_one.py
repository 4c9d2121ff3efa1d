"""One single-graph rollout (fixture, repeats) in the current MD_DF mode; prints the sequence
length, kernel ms and the library's error on failure."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine
W = engine.load_weights(engine.DEFAULT_UNIT)
name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
e = _lib.Engine(W)
e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
for r in range(reps):
    e.reset()
    try:
        out = e.rollout()
    except Exception as ex:
        print(f"{name} MD_DF={os.environ.get('MD_DF', '1')} rep {r}: FAILED {ex}", flush=True)
        sys.exit(1)
    print(f"{name} MD_DF={os.environ.get('MD_DF', '1')} rep {r}: {len(out[0][0])} removals, {e.last_timing()[0]:.3f} ms; "
          f"golden {len(z['seq'])}, equal {list(out[0][0]) == list(z['seq'])}", flush=True)
e.close()
