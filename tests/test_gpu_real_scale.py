"""testReal at the reference's real sizes (BASELINE.json configs[3]).

The reference's real multiplex files are absent; mdcommunity_amd.synth writes an N = 18 000
two-layer file shaped like homo_genetic_multiplex (N = 18 222, heavy-tailed degrees, hubs of
degree ~1 100, nodes missing from a layer, duplicate edges and self-loops for the reader to
drop).  It is read through the drop-in reader (MultiDismantler.read_multiplex, networkx edge
order) and rolled out on the GPU with the environment in HBM (the graph is far beyond one
workgroup's LDS), unit and degree cost, stepRatio 0 and 0.01 (180 removals per prediction
through the host hand-shake).  Checked against the oracle:
* MvcEnv.s0's max_rank and Q at s0 (within 1e-5);
* the LMCC after removal k of the device's own sequence for the first 12 removals (the
  oracle environment stepped along it) and at sampled later k (the mutual-LMCC fixed point of
  the graph without the first k + 1 removed nodes, computed from scratch: the fixed point
  only gets finer as nodes are removed, so it does not depend on the path);
* the sequence is a permutation prefix that ends terminal, and with stepRatio 0.01 each
  prediction's picks are the host's np.argsort(-q)[:180] of the device's own Q;
* whole sequences are certified against tests/golden/real_scale_certs.npz
  (tests/golden/make_real_scale_certs.py: the oracle teacher-forced along the device's
  sequences, and the reference itself for the first predictions): LMCC trace and score
  bit-exact at every removal, every pick inside the oracle's near-tie band, Q within 1e-5 of
  the oracle's and of the reference's rows.
"""
import os
import numpy as np
import pytest

from conftest import GOLDEN
from mdcommunity_amd import _lib, agent, engine, graph as mgraph, synth
from oracle import refenv, refmodel

pytestmark = pytest.mark.gpu
N = 18000


@pytest.fixture(scope="module")
def real(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("real") / "real_like_multiplex.edges")
    synth.write_real_like(path, N, seed=0)
    a = agent.MultiDismantler.__new__(agent.MultiDismantler)
    _, gl = agent.MultiDismantler.read_multiplex(a, path, N)
    e0, e1 = np.asarray(gl[0], np.int32), np.asarray(gl[1], np.int32)
    return e0, e1, refenv.RefGraph(N, e0, e1)


def prefix_lmcc(g, seq, k):
    g1, g2 = g.nx_layers()
    cov = [int(a) for a in seq[: k + 1]]
    g1.remove_nodes_from(cov)
    g2.remove_nodes_from(cov)
    return refenv.lmcc_size(refenv.mutual_components(g1, g2, [set(), set()]))


def check_sequence(g, seq, ranks, cost):
    assert len(seq) == len(set(seq.tolist())) > 0
    env = refenv.RefEnv(g, cost)
    for a, r in zip(seq[:12].tolist(), ranks[:12].tolist()):
        assert env.step(int(a)) == int(r)
    rng = np.random.default_rng(1)
    ks = sorted(set(rng.integers(12, len(seq), size=6).tolist()) | {len(seq) - 1})
    for k in ks:
        assert prefix_lmcc(g, seq, k) == int(ranks[k]), k
    # terminal after the last removal: some layer has no alive edge left
    g1, g2 = g.nx_layers()
    g1.remove_nodes_from(seq.tolist())
    g2.remove_nodes_from(seq.tolist())
    refenv.mutual_components(g1, g2, [set(), set()])
    assert g1.number_of_edges() == 0 or g2.number_of_edges() == 0


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cost", ["unit", "degree"])
def test_real_scale_s0_q_and_rollout(real, cost):
    e0, e1, g = real
    deg = cost == "degree"
    ckpt = engine.DEFAULT_DEGREE if deg else engine.DEFAULT_UNIT_REAL
    eng = _lib.Engine(engine.load_weights(ckpt), cost_mode=_lib.MD_COST_DEGREE if deg else _lib.MD_COST_UNIT)
    try:
        nw = None
        if deg:
            gg = mgraph.Graph_test.from_edges(N, e0, e1)
            mgraph.ensure_degree_weights(gg)
            nw = mgraph.node_weight_array([gg])
        eng.load_graphs([(N, e0, e1)], node_w=nw)
        mr = int(eng.reset()[0])
        assert mr == g.max_rank
        q, _, _, _ = eng.predict()
        env = refenv.RefEnv(g, cost)
        q_ref = refenv.predict(refmodel.RefWeights.load(ckpt), g, set(), env.removed, cost)
        live = q_ref != refenv.MASK
        assert np.array_equal(np.isfinite(q), live)
        dq = float(np.max(np.abs(q[live].astype(np.float64) - q_ref[live])))
        assert dq < 1e-5, dq
        eng.reset()
        seq, ranks = eng.rollout()[0]
        check_sequence(g, seq, ranks, cost)
    finally:
        eng.close()


@pytest.mark.timeout(600)
def test_real_scale_step_ratio(real):
    """stepRatio = 0.01 (U/MultiDismantler_torch.py:676-679,725): 180 removals per prediction,
    every prediction answered by the host's np.argsort(-q)[:180] through the hand-shake."""
    e0, e1, g = real
    step = max(int(0.01 * N), 1)
    eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT_REAL))
    rows = []
    base = eng.selector

    def sel(qrow, n_out):  # the default rule, recording each request's row
        rows.append(qrow.copy())
        return base(qrow, n_out)

    try:
        eng.load_graphs([(N, e0, e1)])
        eng.reset()
        q0, _, _, _ = eng.predict()
        eng.reset()
        eng.selector = sel
        seq, ranks = eng.rollout(step=step)[0]
        check_sequence(g, seq, ranks, "unit")
        assert len(rows) == (len(seq) + step - 1) // step
        # the first request is the s0 prediction; every request's picks are its argsort
        assert np.array_equal(np.isfinite(q0), rows[0] > refenv.MASK)
        for t, r in enumerate(rows):
            picks = np.argsort(-r)[:step].tolist()
            assert seq[t * step:(t + 1) * step].tolist() == picks[: len(seq[t * step:(t + 1) * step])], t
    finally:
        eng.close()


Q_TOL = 1e-5  # north_star: Q within 1e-5
CERT_CASES = {  # fixture case: (cost mode, checkpoint, step) as scripts/dump_real_scale.py ran them
    "deg_step1": (_lib.MD_COST_DEGREE, engine.DEFAULT_DEGREE, 1),
    "unit_step1": (_lib.MD_COST_UNIT, engine.DEFAULT_UNIT_REAL, 1),
    "unit_ratio0.01": (_lib.MD_COST_UNIT, engine.DEFAULT_UNIT_REAL, max(int(0.01 * N), 1)),
}


@pytest.fixture(scope="module")
def certs():
    with np.load(os.path.join(GOLDEN, "real_scale_certs.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", list(CERT_CASES))
def test_real_scale_certified_whole_sequence(real, certs, name):
    """C4 at real size (U/MultiDismantler_torch.py:645-709,676-679; D/MultiDismantler_torch.py:
    623-681): the device rollout of the N = 18 000 multiplex is the certified sequence, its LMCC
    trace and score equal the oracle's at every removal (bit-exact), every pick lies in the
    oracle's near-tie band (a pick the oracle ranks below its max -- or, with 180 picks per
    prediction, below its 180th value -- by more than 2 x Q_TOL would be a wrong decision), and
    the device's Q at the first predictions is within Q_TOL of the oracle's and the reference's."""
    e0, e1, g = real
    cost, ckpt, step = CERT_CASES[name]
    c = {k[len(name) + 1:]: v for k, v in certs.items() if k.startswith(name + "_")}
    eng = _lib.Engine(engine.load_weights(ckpt), cost_mode=cost)
    try:
        gg = mgraph.Graph_test.from_edges(N, e0, e1)
        nw = None
        if cost == _lib.MD_COST_DEGREE:
            mgraph.ensure_degree_weights(gg)
            nw = mgraph.node_weight_array([gg])
        eng.load_graphs([(N, e0, e1)], node_w=nw)
        mr = int(eng.reset()[0])
        assert mr == int(c["max_rank"]) == g.max_rank
        seq, ranks = eng.rollout(step=step)[0]
        # the device is deterministic: the certificate is for exactly this sequence
        assert seq.tolist() == c["seq"].tolist()
        assert ranks.tolist() == c["ranks"].tolist() == c["oracle_ranks"].tolist()
        score = 0.0
        if cost == _lib.MD_COST_DEGREE:  # D/mvc_env.py:127-134
            tw0, tw1 = sum(gg.weights[0].values()), sum(gg.weights[1].values())
            for a, r in zip(seq.tolist(), ranks.tolist()):
                score += -1 * (-int(r) / (mr) * (gg.weights[0][a] / tw0 + gg.weights[1][a] / tw1) / 2.0)
        else:  # U/mvc_env.py:86,133-137
            for r in ranks.tolist():
                score += -1 * (-float(r) / (mr * float(N)))
        assert score == float(c["oracle_score"])
        # every pick inside the oracle's near-tie band
        band = np.repeat(c["kth"] if step > 1 else c["qmax"], step)[:len(seq)]
        margin = band - c["qpick"]
        assert float(np.max(margin)) <= 2 * Q_TOL, (int(np.argmax(margin)), float(np.max(margin)))
        if step == 1:
            # and exactly the oracle's arg-max wherever the oracle's top-2 gap leaves no doubt
            clear = c["gap"] > 2 * Q_TOL
            assert np.all(margin[clear] == 0.0)
        # Q rows, teacher-forced along the sequence: oracle (first Q_ROWS predictions) and the
        # reference itself (first predictions)
        eng.reset()
        dq_o = dq_r = 0.0
        for t in range(len(c["qrows"])):
            q, _, _, _ = eng.predict()
            live = np.isfinite(q)
            for rows, which in ((c["qrows"], "o"), (c["refrows"], "r")):
                if t < len(rows):
                    ref = rows[t].astype(np.float64)
                    assert np.array_equal(live, ref != np.float32(refenv.MASK)), (which, t)
                    d = float(np.max(np.abs(q[live].astype(np.float64) - ref[live])))
                    if which == "o":
                        dq_o = max(dq_o, d)
                    else:
                        dq_r = max(dq_r, d)
            for a in seq[t * step:(t + 1) * step]:
                eng.step(np.asarray([a], np.int32))
        assert dq_o < Q_TOL and dq_r < Q_TOL, (dq_o, dq_r)
    finally:
        eng.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["deg_step1", "unit_step1"])
def test_real_scale_deep_predictions_match_reference(real, certs, name):
    """Deep predictions at real size (U/MultiDismantler_torch.py:711-736,759-784; D/...:683-706):
    the device's Q rows at predictions 40, 80, 120, 158 (unit cost also 177, its last) of the
    certified sequence, teacher-forced, are within Q_TOL of the REFERENCE's own rows
    (tests/golden/real_scale_deep.npz, tests/golden/make_real_scale_deep.py), with the same mask."""
    e0, e1, g = real
    cost, ckpt, step = CERT_CASES[name]
    with np.load(os.path.join(GOLDEN, "real_scale_deep.npz")) as z:
        idx, ref = z[f"{name}_idx"], z[f"{name}_ref"]
    seq = certs[f"{name}_seq"]
    eng = _lib.Engine(engine.load_weights(ckpt), cost_mode=cost)
    try:
        nw = None
        if cost == _lib.MD_COST_DEGREE:
            gg = mgraph.Graph_test.from_edges(N, e0, e1)
            mgraph.ensure_degree_weights(gg)
            nw = mgraph.node_weight_array([gg])
        eng.load_graphs([(N, e0, e1)], node_w=nw)
        eng.reset()
        want = {int(t): k for k, t in enumerate(idx.tolist())}
        dq = 0.0
        for t in range(int(idx.max()) + 1):
            if t in want:
                q, _, _, _ = eng.predict()
                r = ref[want[t]].astype(np.float64)
                live = np.isfinite(q)
                assert np.array_equal(live, r != np.float32(refenv.MASK)), t
                dq = max(dq, float(np.max(np.abs(q[live].astype(np.float64) - r[live]))))
            eng.step(np.asarray([seq[t]], np.int32))
        assert dq < Q_TOL, dq
    finally:
        eng.close()
