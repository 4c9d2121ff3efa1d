#!/usr/bin/env python3
"""Dump the GPU's rollouts of the testReal-sized graph (GPU box only) for the C4 certificates.

The N = 18 000 two-layer multiplex of tests/test_gpu_real_scale.py (mdcommunity_amd.synth seed 0,
read through the drop-in reader) rolled out by the device in the three testReal settings:
degree cost stepRatio 0 (D/testReal.py), unit cost stepRatio 0 and stepRatio 0.01
(U/testReal.py, 180 removals per prediction).  Per case: the sequence, the LMCC trace, max_rank
and the device's Q rows of the first 20 predictions (md_predict teacher-forced along the
sequence).  Output ``gpurun_out/real_scale_traj.npz``; tests/golden/make_real_scale_certs.py
turns it into the committed fixture (the oracle, and for the first predictions the reference
itself, teacher-forced along these sequences).
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, agent, engine, graph as mgraph, synth  # noqa: E402

N = 18000
CASES = {  # name: (cost mode, checkpoint, step)
    "deg_step1": (_lib.MD_COST_DEGREE, engine.DEFAULT_DEGREE, 1),
    "unit_step1": (_lib.MD_COST_UNIT, engine.DEFAULT_UNIT_REAL, 1),
    "unit_ratio0.01": (_lib.MD_COST_UNIT, engine.DEFAULT_UNIT_REAL, max(int(0.01 * N), 1)),
}
Q_ROWS = 20


def real_edges():
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "real_like_multiplex.edges")
        synth.write_real_like(path, N, seed=0)
        a = agent.MultiDismantler.__new__(agent.MultiDismantler)
        _, gl = agent.MultiDismantler.read_multiplex(a, path, N)
    return np.asarray(gl[0], np.int32), np.asarray(gl[1], np.int32)


def main():
    e0, e1 = real_edges()
    out = {"edges0": e0, "edges1": e1}
    for name, (cost, ckpt, step) in CASES.items():
        eng = _lib.Engine(engine.load_weights(ckpt), cost_mode=cost)
        nw = None
        if cost == _lib.MD_COST_DEGREE:
            g = mgraph.Graph_test.from_edges(N, e0, e1)
            mgraph.ensure_degree_weights(g)
            nw = mgraph.node_weight_array([g])
        eng.load_graphs([(N, e0, e1)], node_w=nw)
        mr = int(eng.reset()[0])
        seq, ranks = eng.rollout(step=step)[0]
        # the device's Q at the first predictions, teacher-forced along its own sequence
        eng.reset()
        rows = []
        for t in range(min(Q_ROWS, -(-len(seq) // step))):
            q, _, _, _ = eng.predict()
            rows.append(q.copy())
            for a in seq[t * step:(t + 1) * step]:
                eng.step(np.asarray([a], np.int32))
        eng.close()
        out[f"{name}_seq"] = seq
        out[f"{name}_ranks"] = ranks
        out[f"{name}_max_rank"] = np.int32(mr)
        out[f"{name}_step"] = np.int32(step)
        out[f"{name}_q"] = np.asarray(rows, np.float32)
        print(name, "removals", len(seq), "max_rank", mr, "predictions", -(-len(seq) // step), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "real_scale_traj.npz"), **out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
