#!/usr/bin/env python3
"""Golden stdout of the reference's inference harness, made by running the reference here.

The drop-in must print what the reference prints (a testReal log is the user-visible record
of a run): ``MultiDismantler.__init__`` (``U/MultiDismantler_torch.py:107,124``), ``LoadModel``
(``:797``), ``Evaluate`` (``:566``), ``EvaluateRealData`` (``:674,691``) and ``GetSolution``'s
``Iteration:%d`` once per prediction (``:721``; degree cost ``D/MultiDismantler_torch.py:544,
639,692``).  Same import method and shims as ``make_golden.py``; one process per variant
(both variants use the same module names).  Written per case as ``stdout_<case>.txt``: the
captured lines with the model path replaced by ``<MODEL>`` and the CUDA flag of this
container (no GPU) by ``<CUDA>``.  tqdm writes to stderr and is not part of it.

Usage: ``python tests/golden/make_stdout_golden.py``.
"""
import contextlib
import io
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (helpers only)


def _capture(fn):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = fn()
    return buf.getvalue(), out


def _clean(txt, model):
    lines = txt.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    out = []
    for ln in lines:
        ln = ln.replace(model, "<MODEL>")
        if ln.startswith("CUDA: "):
            ln = "CUDA: <CUDA>"
        out.append(ln)
    return out


def run_variant(variant):
    if variant == "unit":
        M, G, GMM, _ = mg.load_unit_reference()
        vdir, ckpt = mg.UNIT_DIR, mg.UNIT_CKPT
    else:
        mg.install_shims()
        vdir = os.path.join(mg.REF_CODE, "MultiDismantler_degree_cost")
        sys.path.insert(0, vdir)
        import MultiDismantler_torch as M  # noqa: E402
        ckpt = "./models/nrange_30_50_iter_100000.ckpt"
    model = os.path.join(vdir, ckpt)
    cases = {}
    txt, agent = _capture(M.MultiDismantler)
    cases["init"] = _clean(txt, model)
    txt, _ = _capture(lambda: agent.LoadModel(model))
    cases["loadmodel"] = _clean(txt, model)
    with tempfile.TemporaryDirectory() as tmp:
        root = os.path.join(tmp, "r")
        work = os.path.join(root, "a", "b")
        real_dir = os.path.join(root, "data", "real")
        os.makedirs(work, exist_ok=True)
        os.makedirs(real_dir, exist_ok=True)
        with open(os.path.join(HERE, "synth_multiplex.edges")) as f:
            body = f.read()
        with open(os.path.join(real_dir, "synth_multiplex.edges"), "w") as f:
            f.write(body)
        # testSynthetic: Evaluate over the committed N=32 data_g graphs
        syn = np.load(os.path.join(HERE, "synthetic_data_g.npz" if variant == "unit" else "synthetic_deg_data_g.npz"))
        d = os.path.join(root, "data", "synthetic", "data_g", "syn_32")
        os.makedirs(d, exist_ok=True)
        for i in range(20):
            for l in (1, 2):
                e = syn[f"n32_g{i}_e{l - 1}"]
                a = np.zeros((32, 32))
                a[e[:, 0], e[:, 1]] = 1
                a[e[:, 1], e[:, 0]] = 1
                np.save(os.path.join(d, f"adj{l}_{i}.npy"), a)
        save = os.path.join(tmp, "out")
        os.makedirs(save, exist_ok=True)
        here = os.getcwd()
        os.chdir(work)
        try:
            txt, _ = _capture(lambda: agent.Evaluate(None, "32", "data_g", model))
            cases["evaluate_32"] = _clean(txt, model)
            ratios = (0, 0.1) if variant == "unit" else (0,)
            for r in ratios:
                txt, _ = _capture(lambda: agent.EvaluateRealData(None, "synth_multiplex.edges", save, r, 60, (1, 3)))
                cases["testreal_step%g" % r] = _clean(txt, model)
        finally:
            os.chdir(here)
    for name, lines in cases.items():
        with open(os.path.join(HERE, f"stdout_{variant}_{name}.txt"), "w") as f:
            f.write("\n".join(lines) + "\n")
    print(json.dumps({k: len(v) for k, v in cases.items()}))


def main():
    if len(sys.argv) > 1:
        run_variant(sys.argv[1])
        return 0
    for v in ("unit", "degree"):
        subprocess.run([sys.executable, os.path.abspath(__file__), v], check=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
