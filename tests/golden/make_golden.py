#!/usr/bin/env python3
"""Generate the golden parity fixtures by running the REFERENCE implementation here.

Runs only in the build container (``/root/reference`` is absent on the GPU box); its
outputs are committed as small ``.npz`` / text fixtures next to this script.

The reference (``/root/reference/code/MultiDismantler_unit_cost``, "U/") is imported
unmodified with three local shims that do not change arithmetic:

1. ``torch_sparse`` (pinned ``torch-sparse 0.6.18``, ``R/uv.lock:1498``) is not installed;
   a stand-in module provides ``spmm(index, value, m, n, matrix)`` following that
   library's published algorithm: ``index_select(col) * value`` then a sequential
   ``scatter_add`` over ``row`` (torch_scatter's CPU kernel is a sequential loop).
2. ``Tensor.cuda(dev)`` is made a no-op (the reference hard-codes ``.cuda(self.device)``
   at ``U/MultiDismantler_net_graphsage.py:332,350`` and
   ``U/MRGNN/mutil_layer_weight.py:276,288,295``).
3. ``np.mat = np.asmatrix`` (numpy 2.x removed ``np.mat``; ``U/PrepareBatchGraph.py:198``).

Usage: ``python tests/golden/make_golden.py [--quick]``.
"""
import argparse
import json
import os
import random
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_CODE = "/root/reference/code"
UNIT_DIR = os.path.join(REF_CODE, "MultiDismantler_unit_cost")
UNIT_CKPT = "./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt"  # U/testSynthetic.py:19
MASK = -(2147483647 / 2)  # U/MultiDismantler_torch.py:60


def install_shims():
    import torch

    mod = types.ModuleType("torch_sparse")

    def spmm(index, value, m, n, matrix):
        row, col = index[0], index[1]
        mat = matrix if matrix.dim() > 1 else matrix.unsqueeze(-1)
        src = mat.index_select(0, col) * value.unsqueeze(-1)
        out = torch.zeros((m, src.size(1)), dtype=src.dtype)
        return out.scatter_add_(0, row.unsqueeze(-1).expand_as(src), src)

    mod.spmm = spmm
    sys.modules["torch_sparse"] = mod
    torch.Tensor.cuda = lambda self, *a, **k: self
    np.mat = np.asmatrix


def load_unit_reference():
    install_shims()
    sys.path.insert(0, UNIT_DIR)
    import MultiDismantler_torch as M  # noqa: E402  (chdirs to UNIT_DIR)
    import graph as G  # noqa: E402
    import GMM  # noqa: E402
    import Mcc  # noqa: E402
    return M, G, GMM, Mcc


def edges_of(g_nx):
    """Reference edge order: networkx ``G.edges()`` iteration (``U/graph.py:76``)."""
    return np.asarray([(int(u), int(v)) for u, v in g_nx.edges()], dtype=np.int32).reshape(-1, 2)


def er_pair(n, seed1, seed2, p=None):
    import networkx as nx
    p = 4.0 / n if p is None else p
    a1 = nx.to_numpy_array(nx.erdos_renyi_graph(n, p, seed=seed1))
    a2 = nx.to_numpy_array(nx.erdos_renyi_graph(n, p, seed=seed2))
    return a1, a2


def gmm_pair(GMM, n, seed):
    random.seed(seed)
    np.random.seed(seed)
    l1, l2 = GMM.GMM(n)
    a1 = np.zeros((n, n))
    a2 = np.zeros((n, n))
    for u, v in l1:
        a1[u, v] = a1[v, u] = 1
    for u, v in l2:
        a2[u, v] = a2[v, u] = 1
    return a1, a2


def pack_rows(rows):
    """Masked float64 Q rows -> float32 with NaN at the mask (lossless: the reference's Q is a
    float32 tensor widened to float64, U/MultiDismantler_torch.py:291-299)."""
    q = np.asarray(rows, dtype=np.float64)
    live = q != MASK
    q32 = np.where(live, q, np.nan).astype(np.float32)
    assert np.array_equal(q32[live].astype(np.float64), q[live]), "Q row is not float32-exact"
    return q32


class Recorder:
    """Wraps the reference agent to record every prediction and environment step (the
    masked Q row of EVERY prediction is kept)."""

    def __init__(self, agent):
        self.agent = agent
        self.reset()
        orig_pred = agent.PredictWithCurrentQNet

        def pred(g_list, covered, remove_edges):
            env = agent.test_env
            g = env.graph
            alive = [g.num_edges[l] - env.numCoveredEdges[l] - len(env.remove_edge[l]) // 2 for l in range(2)]
            out = orig_pred(g_list, covered, remove_edges)
            q = np.asarray(out[0], dtype=np.float64)
            live = q != MASK
            lq = np.sort(q[live])[::-1]
            qmax = lq[0] if lq.size else MASK
            gap = (lq[0] - lq[1]) if lq.size > 1 else np.inf
            ntie = int(np.sum(q[live] == qmax)) if lq.size else 0
            t = len(self.stats)
            self.stats.append((int(live.sum()), alive[0], alive[1], qmax, gap, ntie,
                               env.numCoveredEdges[0], env.numCoveredEdges[1]))
            assert t == len(self.q_rows)
            self.q_rows.append(q.copy())
            return out

        agent.PredictWithCurrentQNet = pred

    def reset(self):
        self.stats = []
        self.q_rows = []


def run_rollout(M, G, agent, rec, a1, a2):
    import networkx as nx
    g1 = nx.from_numpy_array(a1)
    g2 = nx.from_numpy_array(a2)
    g = G.Graph_test(g1, g2)
    agent.InsertGraph(g, is_test=True)
    rec.reset()
    t0 = time.time()
    score, sol, cost = agent.GetSol(0)
    dt = time.time() - t0
    env = agent.test_env
    ranks = [int(round(x * g.max_rank)) for x in env.MaxCCList[1:]]
    rec_out = dict(
        n_nodes=np.int32(g.num_nodes),
        edges0=edges_of(g1), edges1=edges_of(g2),
        max_rank=np.int32(g.max_rank),
        seq=np.asarray([int(a) for a in sol], dtype=np.int32),
        ranks=np.asarray(ranks, dtype=np.int32),
        score=np.float64(score),
        maxcc=np.asarray(env.MaxCCList, dtype=np.float64),
        removed0=np.int32(len(env.remove_edge[0]) // 2),
        removed1=np.int32(len(env.remove_edge[1]) // 2),
        step_stats=np.asarray([s[:3] + s[5:] for s in rec.stats], dtype=np.int64).reshape(-1, 6),
        step_qmax=np.asarray([s[3] for s in rec.stats], dtype=np.float64),
        step_gap=np.asarray([s[4] for s in rec.stats], dtype=np.float64),
        q_all=pack_rows(rec.q_rows).reshape(len(rec.q_rows), g.num_nodes),
        ref_seconds=np.float64(dt),
    )
    agent.ClearTestGraphs()
    return rec_out


def mcc_cases(Mcc, n_cases, rng):
    """Random (graph, covered) states -> reference MCC result (``U/Mcc.py:30-38``)."""
    import networkx as nx
    cases = []
    for c in range(n_cases):
        n = int(rng.integers(8, 120))
        p = float(rng.uniform(1.0, 6.0)) / n
        a1 = nx.to_numpy_array(nx.erdos_renyi_graph(n, p, seed=int(rng.integers(1 << 30))))
        a2 = nx.to_numpy_array(nx.erdos_renyi_graph(n, p, seed=int(rng.integers(1 << 30))))
        g1 = nx.from_numpy_array(a1)
        g2 = nx.from_numpy_array(a2)
        e0, e1 = edges_of(g1), edges_of(g2)
        k = int(rng.integers(0, max(1, n // 4)))
        covered = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        h1, h2 = g1.copy(), g2.copy()
        h1.remove_nodes_from(covered.tolist())
        h2.remove_nodes_from(covered.tolist())
        rem = [set(), set()]
        comps = Mcc.MCC(h1, h2, rem)
        rank = Mcc.find_max_set_length(comps)
        # removed edges as a 0/1 flag over each layer's edge list (either orientation recorded)
        r0 = np.asarray([(int(u), int(v)) in rem[0] for u, v in e0], dtype=np.uint8)
        r1 = np.asarray([(int(u), int(v)) in rem[1] for u, v in e1], dtype=np.uint8)
        label = np.full(n, -1, dtype=np.int32)
        for comp in comps:
            m = min(comp)
            for v in comp:
                label[v] = m
        cases.append(dict(n=n, e0=e0, e1=e1, covered=covered, rank=rank, r0=r0, r1=r1, label=label))
    return cases


def save_cases(path, cases):
    flat = {}
    for i, c in enumerate(cases):
        for k, v in c.items():
            flat[f"c{i}_{k}"] = np.asarray(v)
    flat["n_cases"] = np.int32(len(cases))
    np.savez_compressed(path, **flat)


def synthetic_dataset(GMM, root, sizes, n_graphs, seed0):
    """testSynthetic inputs: ``../../data/synthetic/<type>/syn_<N>/adj{1,2}_<i>.npy`` (U/MultiDismantler_torch.py:570-571)."""
    edges = {}
    for n in sizes:
        d = os.path.join(root, "data", "synthetic", "data_g", f"syn_{n}")
        os.makedirs(d, exist_ok=True)
        for i in range(n_graphs):
            a1, a2 = gmm_pair(GMM, n, seed0 + 1000 * n + i)
            np.save(os.path.join(d, f"adj1_{i}.npy"), a1)
            np.save(os.path.join(d, f"adj2_{i}.npy"), a2)
            edges[f"n{n}_g{i}_e0"] = np.argwhere(np.triu(a1) > 0).astype(np.int32)
            edges[f"n{n}_g{i}_e1"] = np.argwhere(np.triu(a2) > 0).astype(np.int32)
    return edges


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip the N=1000 rollouts")
    args = ap.parse_args()
    M, G, GMM, Mcc = load_unit_reference()
    import torch
    agent = M.MultiDismantler()
    agent.LoadModel(UNIT_CKPT)
    rec = Recorder(agent)
    meta = {"torch": torch.__version__, "numpy": np.__version__, "torch_threads": torch.get_num_threads(),
            "ckpt": "U/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt", "graphs": {}}

    graphs = {"er100": er_pair(100, 1, 2)}
    if not args.quick:
        for s in (0, 1, 2):
            graphs[f"gmm1000_s{s}"] = gmm_pair(GMM, 1000, s)
        graphs["er1000"] = er_pair(1000, 1, 2)
    graphs["gmm200_s7"] = gmm_pair(GMM, 200, 7)
    graphs["er300_dense"] = er_pair(300, 11, 12, p=8.0 / 300)
    for name, (a1, a2) in graphs.items():
        out = run_rollout(M, G, agent, rec, a1, a2)
        np.savez_compressed(os.path.join(HERE, f"rollout_{name}.npz"), **out)
        meta["graphs"][name] = dict(E=[int(len(out["edges0"])), int(len(out["edges1"]))],
                                    removals=int(len(out["seq"])), audc=float(out["score"]),
                                    max_rank=int(out["max_rank"]), ref_seconds=float(out["ref_seconds"]),
                                    tie_steps=int(np.sum(out["step_stats"][:, 3] > 1)))
        print(name, meta["graphs"][name], flush=True)

    rng = np.random.default_rng(20261015)
    save_cases(os.path.join(HERE, "mcc_cases.npz"), mcc_cases(Mcc, 60, rng))

    # testSynthetic end-to-end: Evaluate() over a small data dir (n_test = 20 graphs per size).
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        root = os.path.join(tmp, "r")
        edges = synthetic_dataset(GMM, root, [32, 64], 20, 500)
        np.savez_compressed(os.path.join(HERE, "synthetic_data_g.npz"), **edges)
        work = os.path.join(root, "a", "b")
        os.makedirs(work, exist_ok=True)
        here = os.getcwd()
        os.chdir(work)
        res = {}
        for n in (32, 64):
            sm, ss, tm, ts, cm = agent.Evaluate(None, str(n), "data_g", os.path.join(UNIT_DIR, UNIT_CKPT))
            res[str(n)] = dict(line="%.4f±%.2f," % (sm, ss), score_mean=float(sm), score_std=float(ss),
                               cost_mean=float(cm))
        os.chdir(here)
        meta["synthetic_data_g"] = res
        print("synthetic", res, flush=True)

        # testReal end-to-end on a synthetic multiplex ``layer u v`` file (U/MultiDismantler_torch.py:602-709).
        real_dir = os.path.join(root, "data", "real")
        os.makedirs(real_dir, exist_ok=True)
        a1, a2 = gmm_pair(GMM, 60, 4242)
        b1, _ = er_pair(60, 5, 6, p=3.0 / 60)
        lines = []
        for lay, a in ((1, a1), (2, b1), (3, a2)):
            for u, v in np.argwhere(np.triu(a) > 0):
                lines.append(f"{lay} {u + 1} {v + 1} 1")
        lines.insert(3, "1 7 7 1")  # a self-loop, dropped by read_multiplex (:626-629)
        with open(os.path.join(real_dir, "synth_multiplex.edges"), "w") as f:
            f.write("\n".join(lines) + "\n")
        with open(os.path.join(HERE, "synth_multiplex.edges"), "w") as f:
            f.write("\n".join(lines) + "\n")
        save = os.path.join(tmp, "out")
        os.makedirs(save, exist_ok=True)
        os.chdir(work)
        sol, st, score = agent.EvaluateRealData(None, "synth_multiplex.edges", save, 0, 60, (1, 3))
        os.chdir(here)
        sub = os.path.join(save, "StepRatio_0.0000")
        for fn in sorted(os.listdir(sub)):
            with open(os.path.join(sub, fn)) as f:
                txt = f.read()
            with open(os.path.join(HERE, "testreal_" + fn), "w") as f:
                f.write(txt)
        meta["testreal"] = dict(layers=[1, 3], N=60, removals=len(sol), audc=float(score))
        print("testreal", meta["testreal"], flush=True)

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
