#!/usr/bin/env python3
"""Dump the GPU's own rollout of every golden fixture, and its Q rows teacher-forced along
both its own trajectory and the reference's (GPU box only).

Output ``gpurun_out/gpu_traj.npz``: per fixture ``<name>_seq``, ``<name>_ranks`` (the GPU
rollout), ``<name>_qgpu`` [steps, n] float32 (md_predict along the GPU's own removals, NaN =
masked), ``<name>_qref`` (md_predict along the reference's removals).  The build container
turns these into the committed certification fixtures (tests/golden/make_certificates.py).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, graph as mgraph  # noqa: E402

UNIT = ["er100", "gmm200_s7", "er300_dense", "gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000"]
DEG = ["deg_er100", "deg_gmm200_s7", "deg_gmm1000_s0"]


def forced_rows(eng, seq):
    eng.reset()
    rows = []
    for a in seq:
        q = eng.predict()[0]
        rows.append(np.where(np.isfinite(q), q, np.nan).astype(np.float32))
        lm, term = eng.step(np.array([a], np.int32))
        if term[0]:
            break
    return np.asarray(rows, np.float32)


def main():
    out = {}
    for name in UNIT + DEG:
        z = np.load(os.path.join(ROOT, "tests", "golden", f"rollout_{name}.npz"))
        n = int(z["n_nodes"])
        deg = name.startswith("deg_")
        if deg:
            g = mgraph.Graph_test.from_edges(n, z["edges0"], z["edges1"])
            mgraph.ensure_degree_weights(g)
            eng = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
            eng.load_graphs([(n, z["edges0"], z["edges1"])], node_w=mgraph.node_weight_array([g]))
        else:
            eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
            eng.load_graphs([(n, z["edges0"], z["edges1"])])
        eng.reset()
        seq, ranks = eng.rollout()[0]
        out[f"{name}_seq"] = seq.astype(np.int32)
        out[f"{name}_ranks"] = ranks.astype(np.int32)
        out[f"{name}_qgpu"] = forced_rows(eng, seq)
        out[f"{name}_qref"] = forced_rows(eng, z["seq"])
        k = 0
        while k < min(len(seq), len(z["seq"])) and seq[k] == z["seq"][k]:
            k += 1
        print(f"{name}: {len(seq)} removals (ref {len(z['seq'])}), common prefix {k}", flush=True)
        eng.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "gpu_traj.npz"), **out)


if __name__ == "__main__":
    main()
