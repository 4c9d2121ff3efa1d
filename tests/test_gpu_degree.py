"""Degree-cost variant (D/) on the GPU against the reference's own outputs
(tests/golden/make_golden_degree.py): node inputs [w, 1] from the original degrees, weighted
reward, Solution_ / NormalizedLMCC_ / Cost_ files."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from test_certificates import PINNED_PREFIX, load_cert
from mdcommunity_amd import _lib, engine, graph as mgraph
from mdcommunity_amd.agent_degree import MultiDismantler

pytestmark = pytest.mark.gpu

Q_TOL = 1e-5
MASK = -(2147483647 / 2)
NAMES = ["deg_er100", "deg_gmm200_s7", "deg_gmm1000_s0"]


@pytest.fixture(scope="module")
def agent():
    a = MultiDismantler()
    a.LoadModel("./models/nrange_30_50_iter_100000.ckpt")  # D/testReal.py, D/testSynthetic.py
    return a


def _graph(z):
    g = mgraph.Graph_test.from_edges(int(z["n_nodes"]), z["edges0"], z["edges1"])
    mgraph.ensure_degree_weights(g)
    return g


@pytest.mark.parametrize("name", NAMES)
def test_degree_q_within_tolerance(name):
    z = load_golden(name)
    g = _graph(z)
    eng = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
    eng.load_graphs([(g.num_nodes, g.edges[0], g.edges[1])], node_w=mgraph.node_weight_array([g]))
    assert int(eng.reset()[0]) == int(z["max_rank"])
    steps = [int(t) for t in z["q_steps"]]
    worst = 0.0
    for t in range(max(steps) + 1):
        if t in steps:
            q = eng.predict()[0]
            ref = z["q_rows"][steps.index(t)]
            live = ref != MASK
            assert np.array_equal(np.isfinite(q), live)
            worst = max(worst, float(np.max(np.abs(q[live].astype(np.float64) - ref[live]))))
        eng.step(np.array([z["seq"][t]], np.int32))
    eng.close()
    assert worst < Q_TOL, worst


@pytest.mark.parametrize("name", NAMES)
def test_degree_getsol_matches_reference(agent, name):
    """GetSol: the whole sequence equals the certified one (equal to the reference's up to the
    pinned divergence step at a reference tie / few-ulp gap, tests/test_certificates.py); the
    weighted score (D/mvc_env.py:127-134) and MaxCCList equal the reference's along it, and the
    score equals the reference's own rollout score, unconditionally."""
    z, c = load_golden(name), load_cert(name)
    g = _graph(z)
    agent.InsertGraph(g, is_test=True)
    score, sol, cost = agent.GetSol(0)
    agent.ClearTestGraphs()
    k = PINNED_PREFIX[name]
    assert sol[:k] == z["seq"][:k].tolist()
    assert sol == c["gpu_seq"].tolist()
    assert score == float(c["ref_score_along"])
    assert score == float(z["score"])
    assert np.array_equal(np.asarray(agent.test_env.MaxCCList), c["ref_maxcc_along"])


def test_degree_batch_matches_single(agent):
    zs = [load_golden(n) for n in NAMES]
    single = []
    for z in zs:
        agent.InsertGraph(_graph(z), is_test=True)
        score, sol, _ = agent.GetSol(0)
        agent.ClearTestGraphs()
        single.append((score, sol))
    res = agent.GetSolBatch([_graph(z) for z in zs])
    for (s1, q1), (score, seq, ranks) in zip(single, res):
        assert seq == q1 and score == s1


def test_degree_evaluate_real_data_files(agent, tmp_path):
    """EvaluateRealData (D): Solution_, NormalizedLMCC_, Cost_ byte-identical."""
    real = tmp_path / "data" / "real"
    real.mkdir(parents=True)
    (real / "synth_multiplex.edges").write_text(open(os.path.join(GOLDEN, "synth_multiplex.edges")).read())
    out = tmp_path / "out"
    out.mkdir()
    agent.EvaluateRealData(None, "synth_multiplex.edges", str(out), 0, 60, (1, 3), data_root=str(tmp_path / "data"))
    sub = out / "StepRatio_0.0000"
    for fn in ("Solution_synth_multiplex_13.txt", "NormalizedLMCC_synth_multiplex_13.txt",
               "Cost_synth_multiplex_13.txt"):
        assert (sub / fn).read_text() == open(os.path.join(GOLDEN, "testreal_deg_" + fn)).read(), fn


def test_degree_evaluate_synthetic(agent, tmp_path):
    """Evaluate (D) on the N=32 golden set: result line and mean cost."""
    meta = json.load(open(os.path.join(GOLDEN, "meta_degree.json")))
    z = np.load(os.path.join(GOLDEN, "synthetic_deg_data_g.npz"))  # drawn with D/GMM.py
    n = 32
    d = tmp_path / "data" / "synthetic" / "data_g" / f"syn_{n}"
    d.mkdir(parents=True)
    for i in range(20):
        for l in range(2):
            a = np.zeros((n, n))
            e = z[f"n{n}_g{i}_e{l}"]
            a[e[:, 0], e[:, 1]] = 1
            a[e[:, 1], e[:, 0]] = 1
            np.save(d / f"adj{l + 1}_{i}.npy", a)
    sm, ss, _, _, cm = agent.Evaluate(None, str(n), "data_g", "./models/nrange_30_50_iter_100000.ckpt",
                                      data_root=str(tmp_path / "data"))
    ref = meta["synthetic_data_g"][str(n)]
    assert "%.4f±%.2f," % (sm, ss) == ref["line"]
    assert abs(sm - ref["score_mean"]) < 1e-12
    assert abs(cm - ref["cost_mean"]) < 1e-12
