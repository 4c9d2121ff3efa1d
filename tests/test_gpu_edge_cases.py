"""Edge cases of the graph inputs on the GPU, checked against the oracle: the smallest graph
(K2), graphs whose size straddles a 64-wide wavefront, isolated nodes, a shared hub (exact Q
ties among its leaves), disconnected clusters, layers of different density, and a graph whose
second layer has no edges (terminal at MvcEnv.s0: U/mvc_env.py:128-131, so GetSol makes no
pick, U/MultiDismantler_torch.py:766).  For each: max_rank equals the oracle's; along the
device's own sequence the live set and Q (within 1e-5) equal the oracle's Predict row at
every state, every pick trails the oracle's best Q by at most twice the measured |dQ| (the
device's pick and the oracle's best each carry an error <= |dQ|), the LMCC after
every removal equals the oracle environment's (bit-exact) and so does the AUDC.  One launch of
all cases (more than 16 graphs: the device work queue) gives each case's single-graph rollout;
so does the grid-wide environment step.  The degree-cost variant is checked the same way
(Q, picks, LMCC; its weighted score is the agent's, tests/test_gpu_degree.py).
The inputs are synthetic (seeded here); the oracle is pinned by tests/test_oracle.py."""
import numpy as np
import pytest

from mdcommunity_amd import _lib, engine, graph as mgraph
from oracle import refenv, refmodel

pytestmark = pytest.mark.gpu

Q_TOL = 1e-5
MASK = refenv.MASK


def er_edges(rng, nodes, p):
    nodes = np.asarray(nodes)
    out = []
    for i in range(len(nodes)):
        for j in range(i + 1, len(nodes)):
            if rng.random() < p:
                out.append((int(nodes[i]), int(nodes[j])))
    rng.shuffle(out)
    return np.array(out, np.int32).reshape(-1, 2)


def cases():
    rng = np.random.default_rng(2026)
    star = np.array([(0, v) for v in range(1, 100)], np.int32)
    tree = np.array([(int(rng.integers(0, v)), v) for v in range(1, 130)], np.int32)
    c1, c2 = np.arange(0, 100), np.arange(100, 200)
    return [
        ("k2", 2, np.array([[0, 1]], np.int32), np.array([[0, 1]], np.int32)),
        ("path_triangle", 3, np.array([[0, 1], [1, 2]], np.int32), np.array([[0, 1], [1, 2], [0, 2]], np.int32)),
        ("shared_hub_star", 100, star, star[::-1].copy()),
        ("isolated_nodes", 50, er_edges(rng, range(40), 0.15), er_edges(rng, range(40), 0.12)),
        ("wave_63", 63, er_edges(rng, range(63), 0.08), er_edges(rng, range(63), 0.1)),
        ("wave_65", 65, er_edges(rng, range(65), 0.08), er_edges(rng, range(65), 0.1)),
        ("two_clusters", 200, np.concatenate([er_edges(rng, c1, 0.06), er_edges(rng, c2, 0.05)]),
         np.concatenate([er_edges(rng, c1, 0.05), er_edges(rng, c2, 0.07)])),
        ("tree_vs_dense", 130, tree, er_edges(rng, range(130), 0.2)),
        ("layer1_empty", 20, er_edges(rng, range(20), 0.3), np.zeros((0, 2), np.int32)),
    ]


CASES = cases()


@pytest.fixture(scope="module")
def weights():
    return refmodel.RefWeights.load(engine.DEFAULT_UNIT)


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    yield e
    e.close()


def audc(ranks, max_rank, n):
    s = 0.0
    for r in ranks:
        s += -1 * (-float(r) / (max_rank * float(n)))  # U/mvc_env.py:86,133-137
    return s


def check_along_device_sequence(eng, weights, name, n, e0, e1, cost="unit"):
    """The device's rollout teacher-forced through the oracle (module docstring); returns the
    device's (sequence, LMCC trace)."""
    g = refenv.RefGraph(n, e0, e1)
    env = refenv.RefEnv(g, cost)
    if cost == "degree":
        eng.load_graphs([(n, e0, e1)], node_w=mgraph.node_weight_array([mgraph.Graph_test.from_edges(n, e0, e1)]))
    else:
        eng.load_graphs([(n, e0, e1)])
    mr = int(eng.reset()[0])
    assert mr == g.max_rank, name
    seq, ranks = eng.rollout()[0]
    if env.terminal():
        assert len(seq) == 0, name
        return seq.tolist(), ranks.tolist()
    eng.reset()
    for t, a in enumerate(seq.tolist()):
        assert not env.terminal(), (name, t)
        ref = refenv.predict(weights, g, env.covered, env.removed, cost)
        q = eng.predict()[0].astype(np.float64)
        live = ref != MASK
        assert np.array_equal(np.isfinite(q), live), (name, t)
        dq = float(np.max(np.abs(q[live] - ref[live])))
        assert dq < Q_TOL, (name, t, dq)
        # the pick can only trail the oracle's best by the two Q errors together (its own and
        # the best node's, each <= dq)
        assert ref[live].max() - ref[a] <= 2 * dq, (name, t, ref[live].max() - ref[a], dq)
        lm, _ = eng.step(np.array([a], np.int32))
        r = env.step(a)
        assert int(lm[0]) == r == int(ranks[t]), (name, t)
    assert env.terminal(), name
    if cost == "unit":
        assert audc(ranks, mr, n) == env.score, name
    return seq.tolist(), ranks.tolist()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_edge_case_rollout_against_oracle(eng, weights, case):
    check_along_device_sequence(eng, weights, *case)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_edge_case_degree_cost_against_oracle(case):
    """Degree cost (D/): node inputs [w, 1] with w = deg / maxdeg of the original layers
    (D/graph.py:91-115; none when the initial LMCC is 1, D/graph.py:80-90)."""
    w = refmodel.RefWeights.load(engine.DEFAULT_DEGREE)
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
    try:
        check_along_device_sequence(e, w, *case, cost="degree")
    finally:
        e.close()


def test_edge_cases_grid_wide_step(eng, monkeypatch):
    """The grid-wide environment step (team_env_step; MD_ENV_MODE=0 + MD_VARIANT=64 force it on
    small graphs) on the same graphs: the rollouts equal the default path's."""
    want = []
    for _, n, e0, e1 in CASES:
        eng.load_graphs([(n, e0, e1)])
        eng.reset()
        s, r = eng.rollout()[0]
        want.append((s.tolist(), r.tolist()))
    monkeypatch.setenv("MD_ENV_MODE", "0")
    monkeypatch.setenv("MD_VARIANT", "64")
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        for (name, n, e0, e1), wnt in zip(CASES, want):
            e.load_graphs([(n, e0, e1)])
            assert int(e.reset()[0]) == refenv.RefGraph(n, e0, e1).max_rank, name
            s, r = e.rollout()[0]
            assert (s.tolist(), r.tolist()) == wnt, name
    finally:
        e.close()


def test_edge_cases_in_one_queue_launch(eng):
    graphs = [(n, e0, e1) for _, n, e0, e1 in CASES]
    single = []
    for gr in graphs:
        eng.load_graphs([gr])
        eng.reset()
        s, r = eng.rollout()[0]
        single.append((s.tolist(), r.tolist()))
    batch = graphs * 3  # 27 graphs: more than the 16 a launch runs without the work queue
    eng.load_graphs(batch)
    mr = eng.reset()
    out = eng.rollout()
    for i, (s, r) in enumerate(out):
        k = i % len(graphs)
        assert (s.tolist(), r.tolist()) == single[k], CASES[k][0]
        assert int(mr[i]) == refenv.RefGraph(*graphs[k]).max_rank, CASES[k][0]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_edge_case_multi_pick_rollout(eng, weights, case):
    """step = 3 picks per prediction (the stepRatio path, np.argsort(-q)[:step],
    U/MultiDismantler_torch.py:725): at each prediction the three picks are np.argsort of the
    device's own masked row, each within twice the measured |dQ| of the oracle's third-best Q; picks stop at the
    terminal state inside a group (:726-729); the LMCC after every removal equals the oracle's."""
    name, n, e0, e1 = case
    g = refenv.RefGraph(n, e0, e1)
    env = refenv.RefEnv(g, "unit")
    eng.load_graphs([(n, e0, e1)])
    eng.reset()
    seq, ranks = eng.rollout(step=3)[0]
    seq = seq.tolist()
    eng.reset()
    t = 0
    while t < len(seq):
        assert not env.terminal(), (name, t)
        ref = refenv.predict(weights, g, env.covered, env.removed)
        q = eng.predict()[0].astype(np.float64)
        live = ref != MASK
        assert np.array_equal(np.isfinite(q), live), (name, t)
        dq = float(np.max(np.abs(q[live] - ref[live])))
        assert dq < Q_TOL, (name, t, dq)
        top = np.sort(ref[live])[::-1]
        group = seq[t:t + 3]
        row = np.where(live, q, MASK)  # the masked float64 row the selection sorts (:286-300)
        assert group == np.argsort(-row)[:len(group)].tolist(), (name, t)
        for a in group:
            assert top[min(2, len(top) - 1)] - ref[a] <= 2 * dq, (name, t, a)
            lm, _ = eng.step(np.array([a], np.int32))
            assert int(lm[0]) == env.step(a) == int(ranks[t]), (name, t)
            t += 1
            if env.terminal():
                break
    assert env.terminal() and t == len(seq), name
