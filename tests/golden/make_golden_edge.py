#!/usr/bin/env python3
"""Reference goldens of the edge-case graphs (tests/edge_graphs.py), made by running the
REFERENCE here -- the same method and the same three arithmetic-neutral shims as
``make_golden.py`` -- so that tests/test_gpu_edge_cases.py checks the device against the
reference itself, not only against the oracle.

Each case's adjacency goes through ``networkx.from_numpy_array`` as in ``make_golden.run_rollout``
(``U/graph.py:69-84``), so the fixture records the reference's own edge order (``G.edges()``),
its whole rollout ``GetSol(0)`` (``U/MultiDismantler_torch.py:759-784``; degree cost
``D/MultiDismantler_torch.py:683-706``), every masked Q row, the LMCC trace and the score.  A case
the reference cannot run is recorded with its error text instead.

Usage: ``python tests/golden/make_golden_edge.py unit`` and ``... degree`` (separate processes:
both variants use the same module names).  Writes ``edge_<cost>.npz`` and ``meta_edge.json``.
"""
import json
import os
import sys
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import make_golden as mg  # noqa: E402  (helpers only; it imports nothing from the reference at load)
from edge_graphs import cases  # noqa: E402


def adjacency(n, edges):
    a = np.zeros((n, n))
    for u, v in np.asarray(edges).reshape(-1, 2):
        a[u, v] = a[v, u] = 1
    return a


def main():
    cost = sys.argv[1] if len(sys.argv) > 1 else "unit"
    if cost == "unit":
        M, G, _, _ = mg.load_unit_reference()
        ckpt = mg.UNIT_CKPT
    else:
        import make_golden_degree as mgd
        M, G, _ = mgd.load_degree_reference()
        ckpt = mgd.DEG_CKPT
    import torch
    agent = M.MultiDismantler()
    agent.LoadModel(ckpt)
    rec = mg.Recorder(agent)
    out, meta = {}, {}
    for name, n, e0, e1 in cases():
        try:
            r = mg.run_rollout(M, G, agent, rec, adjacency(n, e0), adjacency(n, e1))
        except Exception as ex:  # recorded, not hidden: the test then keeps the oracle check only
            meta[name] = {"error": "".join(traceback.format_exception_only(type(ex), ex)).strip()}
            print(name, meta[name], flush=True)
            try:
                agent.ClearTestGraphs()
            except Exception:
                pass
            continue
        for k, v in r.items():
            out[f"{name}__{k}"] = v
        meta[name] = dict(E=[int(len(r["edges0"])), int(len(r["edges1"]))], removals=int(len(r["seq"])),
                          audc=float(r["score"]), max_rank=int(r["max_rank"]),
                          tie_steps=int(np.sum(r["step_stats"][:, 3] > 1)) if len(r["step_stats"]) else 0)
        print(name, meta[name], flush=True)
    np.savez_compressed(os.path.join(HERE, f"edge_{cost}.npz"), **out)
    path = os.path.join(HERE, "meta_edge.json")
    allm = json.load(open(path)) if os.path.exists(path) else {}
    allm[cost] = {"torch": torch.__version__, "numpy": np.__version__, "ckpt": ckpt, "cases": meta}
    with open(path, "w") as f:
        json.dump(allm, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
