#!/usr/bin/env python3
"""Deep-prediction certificates at the reference's real size (N = 18 000, BASELINE configs[3]):
the REFERENCE's masked Q rows at sampled predictions far into the rollout, teacher-forced along
the certified device sequences of ``real_scale_certs.npz`` (``make_real_scale_certs.py``), next to
the ORACLE's rows at the same states.

``make_real_scale_certs.py`` pins the oracle to the reference on the first 5 predictions only;
this extends the pin to predictions 40, 80, 120 and 158 (unit cost also 177, its last), where the
residual graph, degrees and LMCC differ most from the start.  The reference is imported exactly as
``make_golden.py`` does (same three arithmetic-neutral shims) and steps its own environment
(``MvcEnv.stepWithoutReward``, ``U/mvc_env.py:74-87``; degree cost ``D/mvc_env.py``) along the
device's picks; ``PredictWithCurrentQNet`` (``U/MultiDismantler_torch.py:263-306``) runs only at the
sampled predictions.

Written: ``real_scale_deep.npz`` ({case}_idx, {case}_ref: reference rows as float32 with the mask
value kept) and the ``deep`` entries of ``meta_real_scale.json`` (reference vs oracle, bit-exact).
Usage: ``python tests/golden/make_real_scale_deep.py`` (a few minutes).
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

N = 18000
CASES = {"deg_step1": "degree", "unit_step1": "unit"}
SAMPLES = {"deg_step1": [40, 80, 120, 158], "unit_step1": [40, 80, 120, 158, 177]}
MASK = -(2147483647 / 2)


def reference_rows(variant, edges_path, seq, samples):
    import make_golden as mg
    if variant == "unit":
        M, G, _, _ = mg.load_unit_reference()
        ckpt = os.path.join(mg.UNIT_DIR, "./models/g0-1_10w_TORCH-Model_GMM_30_50/nrange_30_50_iter_24000.ckpt")
    else:
        mg.install_shims()
        ddir = os.path.join(mg.REF_CODE, "MultiDismantler_degree_cost")
        sys.path.insert(0, ddir)
        import MultiDismantler_torch as M  # noqa: E402
        import graph as G  # noqa: E402
        ckpt = os.path.join(ddir, "./models/nrange_30_50_iter_100000.ckpt")
    agent = M.MultiDismantler()
    agent.LoadModel(ckpt)
    _, graphs = agent.read_multiplex(edges_path, N)
    g = G.Graph_test(graphs[0], graphs[1])
    env = agent.test_env
    env.s0(g)
    want = set(samples)
    rows = []
    t0 = time.time()
    for t, a in enumerate(seq):
        if t in want:
            q = agent.PredictWithCurrentQNet([env.graph], [env.action_list], [env.remove_edge])[0]
            rows.append(np.asarray(q, np.float64))
            print(f"  reference {variant} prediction {t} ({time.time() - t0:.0f} s)", flush=True)
        env.stepWithoutReward(int(a))
    return np.asarray(rows)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--reference":
        variant, edges_path, name, out_path = sys.argv[2:6]
        certs = np.load(os.path.join(HERE, "real_scale_certs.npz"))
        rows = reference_rows(variant, edges_path, certs[f"{name}_seq"].tolist(), SAMPLES[name])
        np.save(out_path, rows)
        return 0
    import torch
    torch.set_num_threads(16)  # as the reference sets (U/MultiDismantler_torch.py:108): MKL blocking follows it
    certs = np.load(os.path.join(HERE, "real_scale_certs.npz"))
    from mdcommunity_amd import synth
    fixture = {}
    mpath = os.path.join(HERE, "meta_real_scale.json")
    meta = json.load(open(mpath))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "real_like_multiplex.edges")
        synth.write_real_like(path, N, seed=0)
        for name, cost in CASES.items():
            seq = certs[f"{name}_seq"]
            assert int(certs[f"{name}_step"]) == 1
            orc = oracle_rows_from_file(path, certs, name, cost)
            rp = os.path.join(td, f"ref_{name}.npy")
            subprocess.run([sys.executable, os.path.abspath(__file__), "--reference", cost, path, name, rp], check=True)
            ref = np.load(rp)
            idx = np.asarray(SAMPLES[name], np.int32)
            assert len(ref) == len(idx) and idx.max() < len(seq)
            o = np.asarray([orc[int(t)] for t in idx])
            live = ref != MASK
            d = float(np.max(np.abs(ref[live] - o[live].astype(np.float64))))
            fixture[f"{name}_idx"] = idx
            fixture[f"{name}_ref"] = ref.astype(np.float32)
            meta["cases"][name]["deep"] = dict(
                predictions=idx.tolist(), ref_vs_oracle_max_abs=d,
                ref_vs_oracle_same_mask=bool(np.array_equal(live, o != np.float32(MASK))),
                ref_vs_oracle_bitexact_f32=bool(np.array_equal(ref.astype(np.float32), o)),
                live_nodes=[int(x) for x in live.sum(axis=1)])
            print(name, meta["cases"][name]["deep"], flush=True)
    np.savez_compressed(os.path.join(HERE, "real_scale_deep.npz"), **fixture)
    with open(mpath, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


def oracle_rows_from_file(path, certs, name, cost):
    """The oracle teacher-forced along the device sequence on the same file the reference reads
    (read through the package's own reader, which the CPU tests pin to read_multiplex)."""
    from mdcommunity_amd import engine, agent as magent
    from oracle import refenv, refmodel
    ckpt = engine.DEFAULT_DEGREE if cost == "degree" else engine.DEFAULT_UNIT_REAL
    w = refmodel.RefWeights.load(ckpt)
    a = magent.MultiDismantler.__new__(magent.MultiDismantler)
    _, gl = magent.MultiDismantler.read_multiplex(a, path, N)
    g = refenv.RefGraph(N, np.asarray(gl[0], np.int32), np.asarray(gl[1], np.int32))
    assert g.max_rank == int(certs[f"{name}_max_rank"])
    env = refenv.RefEnv(g, cost)
    want = set(SAMPLES[name])
    rows = {}
    t0 = time.time()
    for t, a in enumerate(certs[f"{name}_seq"].tolist()):
        if t in want:
            rows[t] = refenv.predict(w, g, env.covered, env.removed, cost).astype(np.float32)
            print(f"  oracle {name} prediction {t} ({time.time() - t0:.0f} s)", flush=True)
        env.step(int(a))
    return rows


if __name__ == "__main__":
    sys.exit(main())
