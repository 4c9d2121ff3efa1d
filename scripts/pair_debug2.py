"""Paired-tile debugging: 18 copies of one graph, admission 1, two tiles per item; per copy the
first predictions' max Q with MD_PAIR=0 / 1, twice each (a race shows as copies that differ)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden
from mdcommunity_amd import _lib, engine

name = sys.argv[1] if len(sys.argv) > 1 else "gmm200_s7"
admit = int(sys.argv[2]) if len(sys.argv) > 2 else 1
z = load_golden(name)
g = (int(z["n_nodes"]), z["edges0"], z["edges1"])
os.environ["MD_VARIANT"] = str((admit << 16) | (2 << 9))
for pair in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("0", "1", "1")):
    os.environ["MD_PAIR"] = pair
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    e.load_graphs([g] * 18)
    e.reset()
    try:
        out = e.rollout()
    except Exception as ex:
        print("PAIR", pair, "error", ex)
        e.close()
        continue
    q0 = [e.trace(i)["qmax"][:3] for i in range(18)]
    print("PAIR", pair, "pred0 qmax per copy:", " ".join("%.7g" % q[0] for q in q0))
    print("        pred1:", " ".join("%.7g" % (q[1] if len(q) > 1 else 0) for q in q0))
    print("        lens:", [len(o[0]) for o in out])
    e.close()
