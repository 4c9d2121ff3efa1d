"""The drop-in surface (agent / env / harnesses) on the GPU against the reference's outputs."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from mdcommunity_amd import graph as mgraph
from mdcommunity_amd.agent import MultiDismantler
from mdcommunity_amd.mvc_env import MvcEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def agent():
    a = MultiDismantler()
    a.LoadModel("./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt")
    return a


def test_getsol_er100(agent):
    z = load_golden("er100")
    g = mgraph.Graph_test.from_edges(100, z["edges0"], z["edges1"])
    agent.InsertGraph(g, is_test=True)
    score, sol, cost = agent.GetSol(0)
    agent.ClearTestGraphs()
    assert sol == z["seq"].tolist()
    assert score == float(z["score"])
    assert cost == len(sol) / 100
    assert np.array_equal(np.asarray(agent.test_env.MaxCCList), z["maxcc"])


def test_env_api(agent):
    z = load_golden("er100")
    g = mgraph.Graph_test.from_edges(100, z["edges0"], z["edges1"])
    env = MvcEnv(50)
    env.s0(g)
    assert g.max_rank == int(z["max_rank"])
    for a in z["seq"]:
        assert not env.isTerminal()
        env.stepWithoutReward(int(a))
    assert env.isTerminal()
    assert env.score == float(z["score"])
    assert env.MaxCCList == z["maxcc"].tolist()
    assert env.covered_set == set(z["seq"].tolist())
    rem = env.remove_edge
    assert len(rem[0]) // 2 == int(z["removed0"]) and len(rem[1]) // 2 == int(z["removed1"])


def test_predict_arbitrary_state(agent):
    """PredictWithCurrentQNet on an explicit (covered, remove_edge) state (Predict :263-302)."""
    z = load_golden("er100")
    g = mgraph.Graph_test.from_edges(100, z["edges0"], z["edges1"])
    env = MvcEnv(50)
    env.s0(g)
    for a in z["seq"][:1]:
        env.stepWithoutReward(int(a))
    cov, rem = list(env.action_list), env.remove_edge
    q = agent.PredictWithCurrentQNet([g], [cov], [rem])[0]
    t = 1
    ref = z["q_rows"][list(z["q_steps"]).index(t)]
    live = ref != -(2147483647 / 2)
    assert np.array_equal(q != -(2147483647 / 2), live)
    assert np.max(np.abs(q[live] - ref[live])) < 1e-5


def test_evaluate_synthetic_matches_reference(agent, tmp_path):
    """Evaluate (testSynthetic harness) on the golden adj{1,2}_i.npy set: the reference's
    result line '%.4f±%.2f,' for N=32 and N=64."""
    import json
    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    z = np.load(os.path.join(GOLDEN, "synthetic_data_g.npz"))
    for n in (32, 64):
        d = tmp_path / "data" / "synthetic" / "data_g" / f"syn_{n}"
        d.mkdir(parents=True)
        for i in range(20):
            for l in range(2):
                a = np.zeros((n, n))
                e = z[f"n{n}_g{i}_e{l}"]
                a[e[:, 0], e[:, 1]] = 1
                a[e[:, 1], e[:, 0]] = 1
                np.save(d / f"adj{l + 1}_{i}.npy", a)
        sm, ss, _, _, cm = agent.Evaluate(None, str(n), "data_g",
                                          "./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt",
                                          data_root=str(tmp_path / "data"))
        ref = meta["synthetic_data_g"][str(n)]
        assert "%.4f±%.2f," % (sm, ss) == ref["line"]
        assert abs(sm - ref["score_mean"]) < 1e-12
        assert abs(cm - ref["cost_mean"]) < 1e-12


def test_evaluate_real_data_matches_reference(agent, tmp_path):
    """EvaluateRealData (testReal harness) on a synthetic `layer u v` file: Soluion_*.txt and
    NormalizedLMCC_*.txt byte-identical to the reference's output."""
    real = tmp_path / "data" / "real"
    real.mkdir(parents=True)
    (real / "synth_multiplex.edges").write_text(open(os.path.join(GOLDEN, "synth_multiplex.edges")).read())
    out = tmp_path / "out"
    out.mkdir()
    agent.EvaluateRealData(None, "synth_multiplex.edges", str(out), 0, 60, (1, 3), data_root=str(tmp_path / "data"))
    sub = out / "StepRatio_0.0000"
    for fn in ("Soluion_synth_multiplex_13.txt", "NormalizedLMCC_synth_multiplex_13.txt"):
        assert (sub / fn).read_text() == open(os.path.join(GOLDEN, "testreal_" + fn)).read(), fn


def test_batch_api_matches_single(agent):
    zs = [load_golden(n) for n in ("er100", "gmm200_s7", "gmm1000_s1")]
    gs = [mgraph.Graph_test.from_edges(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in zs]
    res = agent.GetSolBatch(gs)
    for z, (score, seq, ranks) in zip(zs, res):
        assert score == float(z["score"])


def test_multi_node_step_getsol(agent):
    """GetSol(step=5): np.argsort(-q)[:5] per prediction (U/MultiDismantler_torch.py:769-775),
    answered by the host through the in-kernel hand-shake.  Blocks of 5 match the reference
    exactly; a block whose top-5 Q values hold a tie or near-tie (< 1e-6, where fp32 rounding
    order decides the order inside the block) is compared as a set (the state after the block
    does not depend on the order); checking stops at a block whose 5th/6th gap is ambiguous.
    The ambiguity of each block is read off the reference's recorded top-6 Q values."""
    z = np.load(os.path.join(GOLDEN, "stepratio_gmm200_s7_step5.npz"))
    zg = load_golden("gmm200_s7")
    kinds = []
    for top in z["top6"]:  # the reference's top-6 Q of each prediction
        inner = bool(np.min(-np.diff(top[:5])) < 1e-6)
        boundary = len(top) > 5 and (top[4] - top[5]) < 1e-6
        kinds.append((inner, boundary))
    g = mgraph.Graph_test.from_edges(int(zg["n_nodes"]), zg["edges0"], zg["edges1"])
    agent.InsertGraph(g, is_test=True)
    score, sol, _ = agent.GetSol(0, step=5)
    agent.ClearTestGraphs()
    ref = z["seq"].tolist()
    checked = 0
    for b, (inner, boundary) in enumerate(kinds):
        if boundary:
            break  # which nodes make the block is itself an fp32-rounding decision
        blk_ref, blk = ref[5 * b:5 * b + 5], sol[5 * b:5 * b + 5]
        if inner:
            assert set(blk) == set(blk_ref), b
        else:
            assert blk == blk_ref, b
        checked += 1
    assert checked >= 2
    if not any(i or bd for i, bd in kinds):
        assert score == float(z["score"])


def test_step_ratio_evaluate_real_data(agent, tmp_path):
    """EvaluateRealData with stepRatio 0.1 (step = 6 nodes per prediction): files
    byte-identical to the reference's."""
    real = tmp_path / "data" / "real"
    real.mkdir(parents=True)
    (real / "synth_multiplex.edges").write_text(open(os.path.join(GOLDEN, "synth_multiplex.edges")).read())
    out = tmp_path / "out"
    out.mkdir()
    agent.EvaluateRealData(None, "synth_multiplex.edges", str(out), 0.1, 60, (1, 3), data_root=str(tmp_path / "data"))
    sub = out / "StepRatio_0.1000"
    for fn in ("Soluion_synth_multiplex_13.txt", "NormalizedLMCC_synth_multiplex_13.txt"):
        assert (sub / fn).read_text() == open(os.path.join(GOLDEN, "testreal_step0.1_" + fn)).read(), fn
