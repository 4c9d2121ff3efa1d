"""Batched prefixes in the grid-wide environment step (md_env.h team_prefix_step, MD_PREFIX):
a prediction's picks (stepRatio > 0: np.argsort(-q)[:step], U/MultiDismantler_torch.py:
725-735) are applied as independent prefix fixed points, one per workgroup, instead of one
cascade after another (tests/test_prefix_states.py: the property it rests on, on the oracle).

MD_ENV_MODE=0 + MD_VARIANT=64 force the grid-wide step on graphs that fit LDS; MD_PREFIX=k takes
batches of at least k actions that way (0: the sequential loop).  Rollouts with several picks
per prediction must be identical -- sequence, LMCC trace -- and leave the identical state
(covered set, removed edges per layer, covered / pruned counters), including batches cut short
by a terminal prefix, batches longer than the launch's workgroups (chunks), and picks of
nodes without alive edges; the LMCC trace is checked against the oracle environment stepped
along the device's sequence (U/mvc_env.py:74-87, U/Mcc.py:30-38)."""
import numpy as np
import pytest

from conftest import load_golden
from mdcommunity_amd import _lib, engine

pytestmark = pytest.mark.gpu

CASES = [("er100", 3), ("er100", 20), ("gmm200_s7", 5), ("er300_dense", 9), ("gmm1000_s0", 16), ("er1000", 64)]


def run(monkeypatch, prefix, name, step, graph=None, degree=False):
    monkeypatch.setenv("MD_ENV_MODE", "0")
    monkeypatch.setenv("MD_VARIANT", "64")
    monkeypatch.setenv("MD_PREFIX", str(prefix))
    if graph is None:
        z = load_golden(name)
        graph = (int(z["n_nodes"]), z["edges0"], z["edges1"])
    n = graph[0]
    nw = None
    if degree:
        from mdcommunity_amd import graph as mgraph
        gg = mgraph.Graph_test.from_edges(n, graph[1], graph[2])
        mgraph.ensure_degree_weights(gg)
        nw = mgraph.node_weight_array([gg])
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE if degree else engine.DEFAULT_UNIT),
                    cost_mode=_lib.MD_COST_DEGREE if degree else _lib.MD_COST_UNIT)
    try:
        e.load_graphs([graph], node_w=nw)
        mr = int(e.reset()[0])
        seq, ranks = e.rollout(step=step)[0]
        served = e.host_requests()
        cov, r0, r1, cnt = e.get_state(0)
        return mr, seq.copy(), ranks.copy(), (cov.tobytes(), r0.tobytes(), r1.tobytes(), cnt.tolist()), served
    finally:
        e.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,step", CASES)
def test_prefix_batches_same_rollouts(monkeypatch, name, step):
    from oracle import refenv
    base = run(monkeypatch, 0, name, step)
    pre = run(monkeypatch, 2, name, step)
    assert pre[0] == base[0]
    assert pre[1].tolist() == base[1].tolist(), name
    assert pre[2].tolist() == base[2].tolist(), name
    assert pre[3] == base[3], name
    z = load_golden(name)
    g = refenv.RefGraph(int(z["n_nodes"]), z["edges0"], z["edges1"])
    env = refenv.RefEnv(g, "unit")
    assert [env.step(int(a)) for a in pre[1].tolist()] == pre[2].tolist()
    assert env.terminal()
    cnt = pre[3][3]
    assert [int(cnt[0]), int(cnt[1])] == env.num_covered
    assert [int(cnt[2]), int(cnt[3])] == [len(env.removed[0]) // 2, len(env.removed[1]) // 2]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,step", [("er100", 3), ("gmm1000_s0", 16), ("er1000", 64)])
def test_device_topk_same_rollouts(monkeypatch, name, step):
    """The grid-wide step's stepRatio picks taken on the device when the k largest Q are
    distinct and above the rest (md_kernels.hip device_topk; MD_DEVTOPK=0: every prediction
    through the host's np.argsort) -- identical sequences, LMCC traces and final states, with
    and without the batched prefixes."""
    out = {}
    for dev in ("0", "1"):
        for prefix in (0, 2):
            monkeypatch.setenv("MD_DEVTOPK", dev)
            out[(dev, prefix)] = run(monkeypatch, prefix, name, step)
    ref = out[("0", 0)]
    for key, r in out.items():
        assert r[0] == ref[0] and r[1].tolist() == ref[1].tolist() and r[2].tolist() == ref[2].tolist(), key
        assert r[3] == ref[3], key
    # the device took predictions itself (fewer host requests than predictions)
    preds = -(-len(ref[1]) // step)
    assert out[("0", 0)][4] == preds
    assert out[("1", 0)][4] < preds, (out[("1", 0)][4], preds)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,step", [("deg_gmm200_s7", 5), ("deg_gmm1000_s0", 12)])
def test_prefix_batches_degree_cost(monkeypatch, name, step):
    """Degree cost (D/mvc_env.py:75-134): the environment step is the same cascade, so the
    batched prefixes give the sequential loop's rollouts and states."""
    base = run(monkeypatch, 0, name, step, degree=True)
    pre = run(monkeypatch, 2, name, step, degree=True)
    for a, b in zip(base[:4], pre[:4]):
        assert (a.tolist() if hasattr(a, "tolist") else a) == (b.tolist() if hasattr(b, "tolist") else b), name


@pytest.mark.timeout(300)
def test_prefix_batches_edge_graphs(monkeypatch):
    """The edge-case graphs (tests/edge_graphs.py: K2, a shared-hub star, isolated nodes, 63 / 65
    nodes, two clusters, a tree against a dense layer, an empty second layer) with 3 and 7 picks
    per prediction: batched prefixes == the sequential loop (sequence, LMCC trace, final state)."""
    from edge_graphs import cases
    for name, n, e0, e1 in cases():
        for step in (3, 7):
            base = run(monkeypatch, 0, name, step, graph=(n, e0, e1))
            pre = run(monkeypatch, 2, name, step, graph=(n, e0, e1))
            assert base[0] == pre[0], name
            assert base[1].tolist() == pre[1].tolist() and base[2].tolist() == pre[2].tolist(), (name, step)
            assert base[3] == pre[3], (name, step)
