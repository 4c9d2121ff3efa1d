#!/usr/bin/env python3
"""Certificates for the GPU's removal sequences beyond the reference's first ambiguous step.

Where the reference itself is ambiguous (an exact tie at the max Q, or a top-2 gap of a few
fp32 ulps), the GPU's pick can legitimately differ from the reference's, and from there on the
two rollouts follow different trajectories.  To certify the GPU's WHOLE sequence, this script
runs the REFERENCE (imported here exactly as make_golden.py does, with the same three
arithmetic-neutral shims) teacher-forced along the GPU's own removal sequence:

    env = reference MvcEnv;  env.s0(g)
    for a in gpu_seq:  q_t = reference PredictWithCurrentQNet(state_t);  env.stepWithoutReward(a)

and records the reference's masked Q row at every GPU state (float32, NaN = masked: lossless),
the reference's LMCC after every GPU removal and its AUDC of the GPU's sequence.
``tests/test_certificates.py`` (CPU) and ``tests/test_gpu_parity.py`` (GPU) then check that
every GPU pick lies in the reference's own near-tie set at that state, that the GPU's LMCC
trace equals the reference's along the same sequence, and that the sequence is pinned.

Input: ``gpurun_out/gpu_traj.npz`` written on the GPU box by ``scripts/dump_gpu_traj.py``
(the GPU sequences are data produced by our library; they are stored in the certificate).

Usage: ``python tests/golden/make_certificates.py --variant unit|degree [--traj PATH]``
(the two variants use the same module names, hence separate processes).
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

UNIT = ["er100", "gmm200_s7", "er300_dense", "gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000"]
DEG = ["deg_er100", "deg_gmm200_s7", "deg_gmm1000_s0"]


def forced(M, G, agent, z, seq):
    """The reference's Q rows, LMCC trace and score along a forced removal sequence
    (GetSol's loop, U/MultiDismantler_torch.py:759-784, with the pick given)."""
    import networkx as nx
    n = int(z["n_nodes"])
    g1, g2 = nx.Graph(), nx.Graph()
    g1.add_nodes_from(range(n))
    g2.add_nodes_from(range(n))
    g1.add_edges_from(z["edges0"].tolist())
    g2.add_edges_from(z["edges1"].tolist())
    g = G.Graph_test(g1, g2)
    assert int(g.max_rank) == int(z["max_rank"])
    env = agent.test_env
    env.s0(g)
    rows = []
    for a in seq:
        assert not env.isTerminal(), "GPU sequence continues past the reference's terminal state"
        q = agent.PredictWithCurrentQNet([g], [env.action_list], [env.remove_edge])[0]
        rows.append(np.asarray(q, dtype=np.float64))
        env.stepWithoutReward(int(a))
    assert env.isTerminal(), "GPU sequence stops before the reference's terminal state"
    ranks = [int(round(x * g.max_rank)) for x in env.MaxCCList[1:]]
    return mg.pack_rows(rows).reshape(len(rows), n), np.asarray(ranks, np.int32), float(env.score), \
        np.asarray(env.MaxCCList, np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", choices=["unit", "degree", "both"], default="both")
    ap.add_argument("--traj", default=os.path.join(HERE, "..", "..", "gpurun_out", "gpu_traj.npz"))
    ap.add_argument("--source", default="", help="provenance string stored in the certificate")
    args = ap.parse_args()
    if args.variant == "both":
        for v in ("unit", "degree"):
            subprocess.run([sys.executable, __file__, "--variant", v, "--traj", args.traj, "--source", args.source],
                           check=True)
        return 0
    tr = np.load(args.traj)
    if args.variant == "unit":
        M, G, _, _ = mg.load_unit_reference()
        agent = M.MultiDismantler()
        agent.LoadModel(mg.UNIT_CKPT)
        names = UNIT
    else:
        import make_golden_degree as mgd
        M, G, _ = mgd.load_degree_reference()
        agent = M.MultiDismantler()
        agent.LoadModel(mgd.DEG_CKPT)
        names = DEG
    summary = {}
    for name in names:
        with np.load(os.path.join(HERE, f"rollout_{name}.npz")) as zz:
            z = {k: zz[k] for k in zz.files}
        seq = tr[f"{name}_seq"].astype(np.int32)
        k = 0
        while k < min(len(seq), len(z["seq"])) and seq[k] == z["seq"][k]:
            k += 1
        rows, ranks, score, maxcc = forced(M, G, agent, z, seq)
        assert np.array_equal(ranks, tr[f"{name}_ranks"]), f"{name}: GPU LMCC trace differs from the reference's"
        q = rows.astype(np.float64)
        margin = np.array([np.nanmax(q[t]) - q[t][seq[t]] for t in range(len(seq))])
        np.savez_compressed(os.path.join(HERE, f"cert_{name}.npz"), gpu_seq=seq, prefix=np.int32(k),
                            ref_q_along=rows, ref_ranks_along=ranks, ref_score_along=np.float64(score),
                            ref_maxcc_along=maxcc, margin=margin, source=np.str_(args.source))
        summary[name] = dict(removals=len(seq), ref_removals=int(len(z["seq"])), prefix=k,
                             max_margin=float(margin.max()), score_along=score, ref_score=float(z["score"]),
                             audc_equal=bool(score == float(z["score"])))
        print(name, summary[name], flush=True)
    path = os.path.join(HERE, "meta_certificates.json")
    meta = json.load(open(path)) if os.path.exists(path) else {}
    meta.update(summary)
    meta["_source"] = args.source
    with open(path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
