"""The drop-in prints what the reference prints: the agent constructor's two lines
(U/MultiDismantler_torch.py:107,124), LoadModel's (:797), Evaluate's model line (:566),
EvaluateRealData's 'testing' / score lines (:674,691) and GetSolution's ``Iteration:%d`` once
per prediction (:721; degree cost D/MultiDismantler_torch.py:544,639,692).  Goldens are the
reference's own stdout captured by tests/golden/make_stdout_golden.py (model path and the CUDA
flag of the container that made them masked)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

UNIT_CKPT = "./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt"
DEG_CKPT = "./models/nrange_30_50_iter_100000.ckpt"


def _golden(variant, case):
    with open(os.path.join(GOLDEN, f"stdout_{variant}_{case}.txt")) as f:
        return f.read().split("\n")[:-1]


def _lines(capsys, model):
    out = capsys.readouterr().out.split("\n")[:-1]
    return ["CUDA: <CUDA>" if ln.startswith("CUDA: ") else ln.replace(model, "<MODEL>") for ln in out]


def _data(tmp_path, variant):
    real = tmp_path / "data" / "real"
    real.mkdir(parents=True)
    (real / "synth_multiplex.edges").write_text(open(os.path.join(GOLDEN, "synth_multiplex.edges")).read())
    syn = np.load(os.path.join(GOLDEN, "synthetic_data_g.npz" if variant == "unit" else "synthetic_deg_data_g.npz"))
    d = tmp_path / "data" / "synthetic" / "data_g" / "syn_32"
    d.mkdir(parents=True)
    for i in range(20):
        for l in range(2):
            a = np.zeros((32, 32))
            e = syn[f"n32_g{i}_e{l}"]
            a[e[:, 0], e[:, 1]] = 1
            a[e[:, 1], e[:, 0]] = 1
            np.save(d / f"adj{l + 1}_{i}.npy", a)
    out = tmp_path / "out"
    out.mkdir()
    return str(tmp_path / "data"), str(out)


@pytest.mark.parametrize("variant", ["unit", "degree"])
def test_stdout_matches_reference(variant, tmp_path, capsys):
    if variant == "unit":
        from mdcommunity_amd.agent import MultiDismantler
        model, ratios = UNIT_CKPT, (0, 0.1)
    else:
        from mdcommunity_amd.agent_degree import MultiDismantler
        model, ratios = DEG_CKPT, (0,)
    root, out = _data(tmp_path, variant)
    capsys.readouterr()
    agent = MultiDismantler()
    got = _lines(capsys, model)
    assert got == _golden(variant, "init")
    assert got[0] == "CUDA: <CUDA>"
    agent.LoadModel(model)
    assert _lines(capsys, model) == _golden(variant, "loadmodel")
    agent.Evaluate(None, "32", "data_g", model, data_root=root)
    assert _lines(capsys, model) == _golden(variant, "evaluate_32")
    for r in ratios:
        agent.EvaluateRealData(None, "synth_multiplex.edges", out, r, 60, (1, 3), data_root=root)
        assert _lines(capsys, model) == _golden(variant, "testreal_step%g" % r), r
