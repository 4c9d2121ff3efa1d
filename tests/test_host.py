"""Host-side logic that needs no GPU: graph containers, multiplex parsing order, paths."""
import os

import networkx as nx
import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from mdcommunity_amd import engine, graph as mgraph
from mdcommunity_amd.agent import MultiDismantler, _edges_in_nx_order


def test_graph_test_edge_order_is_networkx_order():
    rng = np.random.default_rng(0)
    a = (rng.random((40, 40)) < 0.1).astype(float)
    a = np.triu(a, 1)
    a = a + a.T
    g1 = nx.from_numpy_array(a)
    g2 = nx.from_numpy_array(np.roll(np.roll(a, 3, 0), 3, 1))
    g = mgraph.Graph_test(g1, g2)
    assert [tuple(e) for e in g.edges[0].tolist()] == [tuple(map(int, e)) for e in g1.edges()]
    assert g.num_edges == [g1.number_of_edges(), g2.number_of_edges()]


def test_read_multiplex_matches_networkx_insertion_order():
    """read_multiplex (U/MultiDismantler_torch.py:602-635) builds networkx graphs by
    add_edge in file order; our parser reproduces their G.edges() order."""
    path = os.path.join(GOLDEN, "synth_multiplex.edges")
    agent = MultiDismantler.__new__(MultiDismantler)
    _, layers = MultiDismantler.read_multiplex(agent, path, 60)
    # networkx construction as the reference does it
    graphs, cur = [], None
    g = nx.Graph()
    g.add_nodes_from(range(60))
    cur_id = 1
    for line in open(path):
        el = line.strip(" \n").split(" ")
        lid = int(el[0])
        if lid != cur_id:
            graphs.append(g)
            g = nx.Graph()
            g.add_nodes_from(range(60))
            cur_id = lid
        u, v = int(el[1]) - 1, int(el[2]) - 1
        if u == v:
            continue
        g.add_edge(u, v)
    graphs.append(g)
    assert len(layers) == len(graphs) == 3
    for e, gg in zip(layers, graphs):
        assert [tuple(x) for x in e.tolist()] == [tuple(map(int, x)) for x in gg.edges()]


def test_edges_in_nx_order_random():
    rng = np.random.default_rng(3)
    order = []
    seen = set()
    for _ in range(200):
        u, v = rng.integers(0, 30, 2)
        if u == v or (min(u, v), max(u, v)) in seen:
            continue
        seen.add((min(u, v), max(u, v)))
        order.append((int(u), int(v)))
    g = nx.Graph()
    g.add_nodes_from(range(30))
    g.add_edges_from(order)
    assert [tuple(x) for x in _edges_in_nx_order(30, order).tolist()] == [tuple(map(int, e)) for e in g.edges()]


def test_reference_checkpoint_paths_resolve():
    for (var, key), (npz, cost) in engine.KNOWN_CKPTS.items():
        assert engine.resolve_model("./" + key).endswith(npz)
        assert engine.resolve_model("./" + key, cost).endswith(npz)
        assert engine.resolve_model(f"/somewhere/code/{var}/{key}", cost).endswith(npz)
    # the degree checkpoint's file name under another variant directory is not it
    for bad in ("/x/MultiDismantler_unit_cost/models/nrange_30_50_iter_100000.ckpt",
                "/x/CEMultiDismantler/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt",
                "elsewhere/nrange_30_50_iter_100000.ckpt", "./models/unknown.ckpt"):
        with pytest.raises(FileNotFoundError):
            engine.resolve_model(bad)
    # a checkpoint of the other cost model is refused, by reference path or shipped file
    with pytest.raises(ValueError):
        engine.resolve_model("./models/nrange_30_50_iter_100000.ckpt", engine._lib.MD_COST_UNIT)
    with pytest.raises(ValueError):
        engine.resolve_model(engine.DEFAULT_UNIT, engine._lib.MD_COST_DEGREE)
    assert engine.resolve_model("./models/nrange_30_50_iter_100000.ckpt", engine._lib.MD_COST_DEGREE) == \
        engine.DEFAULT_DEGREE
    assert engine.resolve_model(None, engine._lib.MD_COST_DEGREE) == engine.DEFAULT_DEGREE
    w = engine.load_weights("./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt")
    assert w.shape == (31205,) and w.dtype == np.float32


def test_degree_weights():
    z = np.load(os.path.join(GOLDEN, "rollout_er100.npz"))
    g = mgraph.Graph_test.from_edges(100, z["edges0"], z["edges1"])
    w = mgraph.degree_weights(g)
    d = np.bincount(z["edges0"].reshape(-1), minlength=100)
    assert np.allclose(w[0], d / d.max())
