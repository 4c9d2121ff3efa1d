#!/usr/bin/env python3
"""Reference certificates for C3/C5 batch seeds beyond 0-2.

For each chosen GMM N=1000 seed the REFERENCE (imported as make_golden.py does, with the same
three arithmetic-neutral shims) is run twice here:

* its own rollout, ``GetSol`` (U/MultiDismantler_torch.py:759-784): sequence, LMCC trace, AUDC;
* teacher-forced along the GPU's single-graph sequence of that seed (make_certificates.forced):
  its LMCC after every GPU removal, its AUDC of the GPU's sequence, and per GPU pick the margin
  ``max Q_ref - Q_ref[pick]`` (0 when the GPU took the reference's arg-max; a tiny positive
  margin only inside the reference's own near-tie band).

``tests/test_gpu_batch.py`` then requires, for every certified seed inside a batch launch:
the batch's sequence equals the certified GPU sequence, its LMCC trace equals the reference's
along it, its AUDC equals the reference's bit for bit, and every pick's margin is within
2 x 1e-5 (the Q tolerance of north_star, the pick's and the best node's errors together).

Input: ``gpurun_out/batch_seqs.npz`` (scripts/dump_batch_seqs.py on the GPU box: the GPU's own
sequences are data produced by our library).  Seeds: the longest GPU rollouts among 3..511 (the
C3 tail) and the C5 seeds above 511 the dump holds.  Output: ``batch_certs.npz`` +
``meta_batch_certs.json``.

Usage: ``python tests/golden/make_batch_certs.py [--dump PATH] [--longest 6]``.
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402
import make_certificates as mc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", default=os.path.join(ROOT, "gpurun_out", "batch_seqs.npz"))
    ap.add_argument("--longest", type=int, default=6)
    args = ap.parse_args()
    d = np.load(args.dump)
    seeds_all = d["seeds"].tolist()
    cand = [s for s in seeds_all if 3 <= s < 512]
    cand.sort(key=lambda s: (-len(d[f"s{s}_seq"]), s))
    seeds = sorted(cand[:args.longest]) + [s for s in seeds_all if s >= 512]
    M, G, GMM, _ = mg.load_unit_reference()
    agent = M.MultiDismantler()
    agent.LoadModel(mg.UNIT_CKPT)
    rec = mg.Recorder(agent)
    sys.path.insert(0, ROOT)
    from mdcommunity_amd import gmm  # the build's own generator: must give the reference's graphs
    out, meta = {"seeds": np.asarray(seeds, np.int32)}, {"seeds": {}}
    for s in seeds:
        a1, a2 = mg.gmm_pair(GMM, 1000, s)
        own = mg.run_rollout(M, G, agent, rec, a1, a2)
        e0, e1 = gmm.gmm_pair(1000, seed=s)
        assert np.array_equal(own["edges0"], e0) and np.array_equal(own["edges1"], e1), s
        gseq = d[f"s{s}_seq"]
        assert int(d[f"s{s}_max_rank"]) == int(own["max_rank"]), s
        z = {"n_nodes": own["n_nodes"], "edges0": own["edges0"], "edges1": own["edges1"], "max_rank": own["max_rank"]}
        rows, ranks_along, score_along, _ = mc.forced(M, G, agent, z, gseq.tolist())
        q = rows.astype(np.float64)
        margin = np.array([np.nanmax(q[t]) - q[t][a] for t, a in enumerate(gseq.tolist())])
        k = 0
        while k < min(len(gseq), len(own["seq"])) and gseq[k] == own["seq"][k]:
            k += 1
        out[f"s{s}_gpu_seq"] = gseq.astype(np.int32)
        out[f"s{s}_ref_ranks_along"] = ranks_along
        out[f"s{s}_ref_score_along"] = np.float64(score_along)
        out[f"s{s}_margin"] = margin
        out[f"s{s}_ref_seq"] = own["seq"]
        out[f"s{s}_ref_score"] = own["score"]
        out[f"s{s}_max_rank"] = own["max_rank"]
        meta["seeds"][str(s)] = dict(removals=int(len(gseq)), ref_removals=int(len(own["seq"])), common_prefix=k,
                                     audc_ref=float(own["score"]), audc_along=float(score_along),
                                     max_margin=float(margin.max()), gpu_ranks_equal=bool(
                                         np.array_equal(d[f"s{s}_ranks"], ranks_along)))
        print(s, meta["seeds"][str(s)], flush=True)
    np.savez_compressed(os.path.join(HERE, "batch_certs.npz"), **out)
    with open(os.path.join(HERE, "meta_batch_certs.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
