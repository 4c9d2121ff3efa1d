"""The CPU oracle against the golden vectors produced by running the reference itself
(tests/golden/make_golden.py): pins the restatement used as the parity checker."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import refenv, refmodel
from mdcommunity_amd import engine

MASK = refenv.MASK


@pytest.fixture(scope="module")
def weights():
    torch.set_num_threads(16)  # as the reference (U/MultiDismantler_torch.py:108)
    return refmodel.RefWeights.load(engine.DEFAULT_UNIT)


@pytest.fixture(scope="module")
def weights_degree():
    torch.set_num_threads(16)
    return refmodel.RefWeights.load(engine.DEFAULT_DEGREE)


@pytest.mark.parametrize("name", ["er100", "gmm200_s7", "er300_dense", "gmm1000_s0", "gmm1000_s1", "gmm1000_s2",
                                  "er1000", "deg_er100", "deg_gmm200_s7", "deg_gmm1000_s0"])
def test_rollout_matches_reference(weights, weights_degree, name):
    """Unit cost (U/) and degree cost (D/, fixtures of make_golden_degree.py)."""
    z = load_golden(name)
    cost = "degree" if name.startswith("deg_") else "unit"
    w = weights_degree if cost == "degree" else weights
    g = refenv.RefGraph(int(z["n_nodes"]), z["edges0"], z["edges1"])
    assert g.max_rank == int(z["max_rank"])
    rows = {}
    score, seq, ranks, maxcc = refenv.rollout(w, g, on_predict=lambda t, q, env: rows.__setitem__(t, q), cost=cost)
    assert seq == z["seq"].tolist()
    assert ranks == z["ranks"].tolist()
    assert score == float(z["score"])  # AUDC, bit-exact float64
    assert np.array_equal(np.asarray(maxcc), z["maxcc"])
    for i, t in enumerate(z["q_steps"]):
        q = rows[int(t)]
        ref = z["q_rows"][i]
        assert np.array_equal(q == MASK, ref == MASK)
        # bit-identical on the build host (same torch/MKL); 1e-6 elsewhere
        assert np.max(np.abs(q - ref)) <= 1e-6


def test_step_statistics(weights):
    """Per-step live-node / alive-edge counts of the oracle match the reference's."""
    z = load_golden("er100")
    g = refenv.RefGraph(int(z["n_nodes"]), z["edges0"], z["edges1"])
    stats = []

    def cb(t, q, env):
        alive = [g.num_edges[l] - env.num_covered[l] - len(env.removed[l]) // 2 for l in range(2)]
        stats.append((int(np.sum(q != MASK)), alive[0], alive[1]))

    refenv.rollout(weights, g, on_predict=cb)
    assert [tuple(s) for s in z["step_stats"][:, :3].tolist()] == stats


def test_mcc_cases_match_reference():
    """Mutual-LMCC cascade of the oracle on random (graph, covered) states vs U/Mcc.py."""
    import networkx as nx
    z = np.load(f"{__import__('conftest').GOLDEN}/mcc_cases.npz")
    for i in range(int(z["n_cases"])):
        n = int(z[f"c{i}_n"])
        e0, e1 = z[f"c{i}_e0"].reshape(-1, 2), z[f"c{i}_e1"].reshape(-1, 2)
        cov = z[f"c{i}_covered"].tolist()
        gs = []
        for e in (e0, e1):
            g = nx.Graph()
            g.add_nodes_from(range(n))
            g.add_edges_from(e.tolist())
            g.remove_nodes_from(cov)
            gs.append(g)
        rem = [set(), set()]
        comps = refenv.mutual_components(gs[0], gs[1], rem)
        assert refenv.lmcc_size(comps) == int(z[f"c{i}_rank"])
        r0 = np.asarray([(int(u), int(v)) in rem[0] for u, v in e0], np.uint8)
        r1 = np.asarray([(int(u), int(v)) in rem[1] for u, v in e1], np.uint8)
        assert np.array_equal(r0, z[f"c{i}_r0"]) and np.array_equal(r1, z[f"c{i}_r1"])


def _edge_goldens(cost):
    import json
    import os
    from conftest import GOLDEN
    with np.load(os.path.join(GOLDEN, f"edge_{cost}.npz")) as z:
        flat = {k: z[k] for k in z.files}
    out = {}
    for k, v in flat.items():
        name, field = k.split("__", 1)
        out.setdefault(name, {})[field] = v
    with open(os.path.join(GOLDEN, "meta_edge.json")) as f:
        return out, json.load(f)[cost]["cases"]


@pytest.mark.parametrize("cost", ["unit", "degree"])
def test_edge_cases_match_reference(weights, weights_degree, cost):
    """The oracle on the edge-case graphs (tests/edge_graphs.py) against the reference's own
    rollouts of them (tests/golden/make_golden_edge.py): max_rank, sequence, LMCC trace and
    (unit cost) AUDC equal, Q rows within 1e-6 (bit-identical on the build host)."""
    gold, meta = _edge_goldens(cost)
    w = weights_degree if cost == "degree" else weights
    assert set(gold) | {k for k, m in meta.items() if "error" in m} == set(meta)
    for name, z in gold.items():
        n = int(z["n_nodes"])
        g = refenv.RefGraph(n, z["edges0"].reshape(-1, 2), z["edges1"].reshape(-1, 2))
        assert g.max_rank == int(z["max_rank"]), name
        rows = {}
        score, seq, ranks, _ = refenv.rollout(w, g, on_predict=lambda t, q, env: rows.__setitem__(t, q), cost=cost)
        assert seq == z["seq"].tolist(), name
        assert ranks == z["ranks"].tolist(), name
        if cost == "unit":
            assert score == float(z["score"]), name
        q_all = z["q_all"].reshape(-1, n).astype(np.float64)
        for t in range(len(q_all)):
            ref = q_all[t]
            live = ~np.isnan(ref)
            assert np.array_equal(rows[t] != MASK, live), (name, t)
            assert np.max(np.abs(rows[t][live] - ref[live])) <= 1e-6, (name, t)
