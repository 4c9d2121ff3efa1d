#!/usr/bin/env python3
"""C4 certificates at the reference's real size (BASELINE configs[3]).

Input: ``gpurun_out/real_scale_traj.npz``, the device's rollouts of the N = 18 000 testReal-shaped
multiplex written on the GPU box by ``scripts/dump_real_scale.py`` (degree cost stepRatio 0, unit
cost stepRatio 0 and 0.01).  Here, in the build container:

* the ORACLE (oracle/refenv.py, the op-for-op restatement) is teacher-forced along each device
  sequence: at every prediction it computes the full masked Q row and records the max, the
  top-2 gap, the oracle Q of each device pick and (stepRatio 0.01) the oracle's step-th and
  (step+1)-th largest values; it steps its own environment along the device's picks, giving
  the LMCC trace and the score with the reference's float64 expressions;
* the REFERENCE itself (imported as make_golden.py does, same three shims; read_multiplex on the
  same ``layer u v`` file) is teacher-forced along the same sequences for the first
  ``REF_PREDICTIONS`` predictions -- its masked Q rows are stored and must equal the oracle's
  (this pins the oracle at N = 18 000, beyond the N <= 1000 goldens).

Written: ``tests/golden/real_scale_certs.npz`` (per case: device sequence and LMCC trace, the
per-prediction oracle summaries, the oracle's LMCC trace and score, the first Q_ROWS oracle Q rows
and the first REF_PREDICTIONS reference Q rows as float32) and ``meta_real_scale.json``.
tests/test_gpu_real_scale.py checks a fresh device rollout against it.

Usage: ``python tests/golden/make_real_scale_certs.py [gpurun_out/real_scale_traj.npz]``.
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
CASES = {"deg_step1": "degree", "unit_step1": "unit", "unit_ratio0.01": "unit"}
Q_ROWS = 20
REF_PREDICTIONS = 5
MASK = -(2147483647 / 2)


def oracle_case(traj, name, cost):
    from mdcommunity_amd import engine
    from oracle import refenv, refmodel
    e0, e1 = traj["edges0"], traj["edges1"]
    seq = traj[f"{name}_seq"].astype(np.int64)
    ranks = traj[f"{name}_ranks"].astype(np.int64)
    step = int(traj[f"{name}_step"])
    ckpt = engine.DEFAULT_DEGREE if cost == "degree" else engine.DEFAULT_UNIT_REAL
    w = refmodel.RefWeights.load(ckpt)
    g = refenv.RefGraph(N, e0, e1)
    assert g.max_rank == int(traj[f"{name}_max_rank"])
    env = refenv.RefEnv(g, cost)
    npred = -(-len(seq) // step)
    qmax, gap, kth, kth1 = (np.zeros(npred) for _ in range(4))
    qpick = np.zeros(len(seq))
    nlive = np.zeros(npred, np.int64)
    rows = []
    k = 0
    t0 = time.time()
    for t in range(npred):
        assert not env.terminal(), t
        q = refenv.predict(w, g, env.covered, env.removed, cost)
        live = q[q != MASK]
        s = np.sort(live)[::-1]
        nlive[t] = len(live)
        qmax[t] = s[0]
        gap[t] = s[0] - s[1] if len(s) > 1 else np.inf
        kth[t] = s[min(step, len(s)) - 1]
        kth1[t] = s[step] if len(s) > step else -np.inf
        if t < Q_ROWS:
            rows.append(q.astype(np.float32))
        for a in seq[t * step:(t + 1) * step]:
            assert not env.terminal()
            qpick[k] = q[int(a)]
            env.step(int(a))
            k += 1
        if t % 20 == 0:
            print(f"  {name} prediction {t}/{npred} ({time.time() - t0:.0f} s)", flush=True)
    assert k == len(seq) and env.terminal()
    oranks = np.asarray(env.ranks, np.int64)
    out = {f"{name}_seq": seq.astype(np.int32), f"{name}_ranks": ranks.astype(np.int32),
           f"{name}_step": np.int32(step), f"{name}_max_rank": np.int32(g.max_rank),
           f"{name}_oracle_ranks": oranks.astype(np.int32), f"{name}_oracle_score": np.float64(env.score),
           f"{name}_qmax": qmax, f"{name}_gap": gap, f"{name}_kth": kth, f"{name}_kth1": kth1,
           f"{name}_qpick": qpick, f"{name}_nlive": nlive, f"{name}_qrows": np.asarray(rows, np.float32)}
    meta = dict(removals=int(len(seq)), predictions=int(npred), step=step, max_rank=int(g.max_rank),
                ranks_equal=bool(np.array_equal(oranks, ranks)), score=float(env.score),
                oracle_seconds=round(time.time() - t0, 1),
                min_gap=float(np.min(gap)),
                # step 1: picks below the oracle's max; step k: picks below the oracle's k-th value
                picks_below_band=int(np.sum(qpick < np.repeat(kth if step > 1 else qmax, step)[:len(seq)])))
    return out, meta


def reference_rows(variant, edges_path, seqs):
    """Run in a subprocess: the reference teacher-forced along `seqs` {name: (seq, step)} for the
    first REF_PREDICTIONS predictions; returns {name: [q rows]}."""
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
    out = {}
    for name, (seq, step) in seqs.items():
        g = G.Graph_test(graphs[0], graphs[1])
        env = agent.test_env
        env.s0(g)
        rows = []
        for t in range(min(REF_PREDICTIONS, -(-len(seq) // step))):
            q = agent.PredictWithCurrentQNet([env.graph], [env.action_list], [env.remove_edge])[0]
            rows.append(np.asarray(q, np.float64))
            for a in seq[t * step:(t + 1) * step]:
                env.stepWithoutReward(int(a))
            print(f"  reference {name} prediction {t}", flush=True)
        out[name] = np.asarray(rows)
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--reference":
        variant, edges_path, traj_path, out_path = sys.argv[2:6]
        traj = np.load(traj_path)
        seqs = {n: (traj[f"{n}_seq"].tolist(), int(traj[f"{n}_step"])) for n, c in CASES.items() if c == variant}
        rows = reference_rows(variant, edges_path, seqs)
        np.savez_compressed(out_path, **rows)
        return 0
    traj_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "real_scale_traj.npz")
    traj = np.load(traj_path)
    import torch
    torch.set_num_threads(16)  # as the reference sets (U/MultiDismantler_torch.py:108)
    from mdcommunity_amd import synth
    fixture, meta = {}, {"N": N, "q_rows": Q_ROWS, "ref_predictions": REF_PREDICTIONS, "cases": {}}
    for name, cost in CASES.items():
        out, m = oracle_case(traj, name, cost)
        fixture.update(out)
        meta["cases"][name] = m
        print(name, m, flush=True)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "real_like_multiplex.edges")
        synth.write_real_like(path, N, seed=0)
        for variant in ("unit", "degree"):
            rp = os.path.join(td, f"ref_{variant}.npz")
            subprocess.run([sys.executable, os.path.abspath(__file__), "--reference", variant, path,
                            os.path.abspath(traj_path), rp], check=True)
            with np.load(rp) as z:
                for name in z.files:
                    ref = z[name]
                    orc = fixture[f"{name}_qrows"][:len(ref)]
                    live = ref != MASK
                    same_mask = bool(np.array_equal(live, orc != np.float32(MASK)))
                    d = float(np.max(np.abs(ref[live] - orc[live].astype(np.float64))))
                    bit = bool(np.array_equal(ref.astype(np.float32), orc))
                    fixture[f"{name}_refrows"] = ref.astype(np.float32)
                    meta["cases"][name].update(ref_predictions=int(len(ref)), ref_vs_oracle_max_abs=d,
                                               ref_vs_oracle_same_mask=same_mask, ref_vs_oracle_bitexact_f32=bit)
                    print(name, "reference vs oracle: max |dQ|", d, "same mask", same_mask, "bit-exact", bit, flush=True)
    np.savez_compressed(os.path.join(HERE, "real_scale_certs.npz"), **fixture)
    with open(os.path.join(HERE, "meta_real_scale.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
