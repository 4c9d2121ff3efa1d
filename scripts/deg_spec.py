import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden
from mdcommunity_amd import _lib, engine, graph as mgraph
z = load_golden("deg_gmm1000_s0")
g = mgraph.Graph_test.from_edges(int(z["n_nodes"]), z["edges0"], z["edges1"])
mgraph.ensure_degree_weights(g)
for v in ("0", "1"):
    os.environ["MD_VARIANT"] = v
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
    e.load_graphs([(g.num_nodes, g.edges[0], g.edges[1])], node_w=mgraph.node_weight_array([g]))
    ts = []
    for _ in range(7):
        e.reset(); out = e.rollout(); ts.append(e.last_timing()[0])
    print("variant", v, "kernel ms", sorted(ts)[3], "removals", len(out[0][0]), "spec hits", e.spec_stats(0), flush=True)
    e.close()
