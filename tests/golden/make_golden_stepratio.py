#!/usr/bin/env python3
"""Golden fixtures of the multi-node step (``stepRatio > 0``: ``np.argsort(-q)[:step]``,
U/MultiDismantler_torch.py:711-736, :664-667), made by running the unit-cost reference here
with the shims of make_golden.py.

* testReal on the committed synth_multiplex.edges with stepRatio 0.1 (step = 6);
* GetSol(gid, step=5) on the gmm200_s7 graph.

Usage: ``python tests/golden/make_golden_stepratio.py``.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def main():
    M, G, GMM, Mcc = mg.load_unit_reference()
    import networkx as nx
    agent = M.MultiDismantler()
    agent.LoadModel(mg.UNIT_CKPT)
    meta = {}
    # GetSol with step 5; the top-6 Q of every prediction (block-order ambiguity)
    top6 = []
    orig_pred = agent.PredictWithCurrentQNet

    def pred(g_list, covered, remove_edges):
        out = orig_pred(g_list, covered, remove_edges)
        top6.append(np.sort(np.asarray(out[0], np.float64))[::-1][:6])
        return out

    agent.PredictWithCurrentQNet = pred
    a1, a2 = mg.gmm_pair(GMM, 200, 7)
    g = G.Graph_test(nx.from_numpy_array(a1), nx.from_numpy_array(a2))
    agent.InsertGraph(g, is_test=True)
    score, sol, cost = agent.GetSol(0, step=5)
    agent.ClearTestGraphs()
    agent.PredictWithCurrentQNet = orig_pred
    np.savez_compressed(os.path.join(HERE, "stepratio_gmm200_s7_step5.npz"),
                        seq=np.asarray([int(a) for a in sol], np.int32), score=np.float64(score),
                        maxcc=np.asarray(agent.test_env.MaxCCList, np.float64),
                        top6=np.asarray(top6, np.float64).reshape(len(top6), -1))
    meta["gmm200_s7_step5"] = dict(removals=len(sol), audc=float(score))
    print(meta, flush=True)
    with tempfile.TemporaryDirectory() as tmp:
        root = os.path.join(tmp, "r")
        work = os.path.join(root, "a", "b")
        real_dir = os.path.join(root, "data", "real")
        os.makedirs(work)
        os.makedirs(real_dir)
        with open(os.path.join(HERE, "synth_multiplex.edges")) as f:
            txt = f.read()
        with open(os.path.join(real_dir, "synth_multiplex.edges"), "w") as f:
            f.write(txt)
        save = os.path.join(tmp, "out")
        os.makedirs(save)
        here = os.getcwd()
        os.chdir(work)
        sol, st, score = agent.EvaluateRealData(None, "synth_multiplex.edges", save, 0.1, 60, (1, 3))
        os.chdir(here)
        sub = os.path.join(save, "StepRatio_0.1000")
        for fn in sorted(os.listdir(sub)):
            with open(os.path.join(sub, fn)) as f:
                body = f.read()
            with open(os.path.join(HERE, "testreal_step0.1_" + fn), "w") as f:
                f.write(body)
        meta["testreal_step0.1"] = dict(removals=len(sol), audc=float(score))
    print(meta, flush=True)
    with open(os.path.join(HERE, "meta_stepratio.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
