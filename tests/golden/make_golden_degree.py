#!/usr/bin/env python3
"""Golden fixtures of the DEGREE-COST variant, made by running the reference here.

Same method as ``make_golden.py`` (same three arithmetic-neutral shims) on
``/root/reference/code/MultiDismantler_degree_cost`` ("D/"): static node inputs
``[deg/maxdeg, 1]`` (``D/PrepareBatchGraph.py:133-136``, weights ``D/graph.py:91-115``),
weighted reward (``D/mvc_env.py:127-134``), checkpoint ``D/models/nrange_30_50_iter_100000.ckpt``
(``D/testSynthetic.py``), testReal files ``Solution_`` / ``NormalizedLMCC_`` / ``Cost_``
(``D/MultiDismantler_torch.py:623-681``).  Runs in a separate process from make_golden.py
because both variants use the same module names.

Usage: ``python tests/golden/make_golden_degree.py``.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (helpers only; it imports nothing from the reference at load)

DEG_DIR = os.path.join(mg.REF_CODE, "MultiDismantler_degree_cost")
DEG_CKPT = "./models/nrange_30_50_iter_100000.ckpt"


def load_degree_reference():
    mg.install_shims()
    sys.path.insert(0, DEG_DIR)
    import MultiDismantler_torch as M  # noqa: E402  (chdirs to DEG_DIR)
    import graph as G  # noqa: E402
    import GMM  # noqa: E402
    return M, G, GMM


def main():
    M, G, GMM = load_degree_reference()
    import torch
    agent = M.MultiDismantler()
    agent.LoadModel(DEG_CKPT)
    rec = mg.Recorder(agent)
    meta = {"torch": torch.__version__, "numpy": np.__version__, "torch_threads": torch.get_num_threads(),
            "ckpt": "D/models/nrange_30_50_iter_100000.ckpt", "graphs": {}}
    graphs = {
        "deg_er100": mg.er_pair(100, 1, 2),
        "deg_gmm200_s7": mg.gmm_pair(GMM, 200, 7),
        "deg_gmm1000_s0": mg.gmm_pair(GMM, 1000, 0),
    }
    for name, (a1, a2) in graphs.items():
        out = mg.run_rollout(M, G, agent, rec, a1, a2)
        np.savez_compressed(os.path.join(HERE, f"rollout_{name}.npz"), **out)
        meta["graphs"][name] = dict(E=[int(len(out["edges0"])), int(len(out["edges1"]))],
                                    removals=int(len(out["seq"])), audc=float(out["score"]),
                                    max_rank=int(out["max_rank"]), ref_seconds=float(out["ref_seconds"]),
                                    tie_steps=int(np.sum(out["step_stats"][:, 3] > 1)))
        print(name, meta["graphs"][name], flush=True)

    with tempfile.TemporaryDirectory() as tmp:
        root = os.path.join(tmp, "r")
        work = os.path.join(root, "a", "b")
        os.makedirs(work, exist_ok=True)
        here = os.getcwd()
        # testSynthetic (degree cost): Evaluate over an N=32 data dir drawn with D's own GMM
        # generator (D/GMM.py differs from U/GMM.py), edges kept as the fixture
        edges = mg.synthetic_dataset(GMM, root, [32], 20, 500)
        np.savez_compressed(os.path.join(HERE, "synthetic_deg_data_g.npz"), **edges)
        os.chdir(work)
        sm, ss, tm, ts, cm = agent.Evaluate(None, "32", "data_g", os.path.join(DEG_DIR, DEG_CKPT))
        os.chdir(here)
        meta["synthetic_data_g"] = {"32": dict(line="%.4f±%.2f," % (sm, ss), score_mean=float(sm),
                                               score_std=float(ss), cost_mean=float(cm))}
        print("synthetic", meta["synthetic_data_g"], flush=True)
        # testReal (degree cost) on the committed synthetic multiplex file
        real_dir = os.path.join(root, "data", "real")
        os.makedirs(real_dir, exist_ok=True)
        with open(os.path.join(HERE, "synth_multiplex.edges")) as f:
            txt = f.read()
        with open(os.path.join(real_dir, "synth_multiplex.edges"), "w") as f:
            f.write(txt)
        save = os.path.join(tmp, "out")
        os.makedirs(save, exist_ok=True)
        os.chdir(work)
        sol, st, score = agent.EvaluateRealData(None, "synth_multiplex.edges", save, 0, 60, (1, 3))
        os.chdir(here)
        sub = os.path.join(save, "StepRatio_0.0000")
        for fn in sorted(os.listdir(sub)):
            with open(os.path.join(sub, fn)) as f:
                body = f.read()
            with open(os.path.join(HERE, "testreal_deg_" + fn), "w") as f:
                f.write(body)
        meta["testreal"] = dict(layers=[1, 3], N=60, removals=len(sol), audc=float(score))
        print("testreal", meta["testreal"], flush=True)

    with open(os.path.join(HERE, "meta_degree.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
