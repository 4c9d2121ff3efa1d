#!/usr/bin/env python3
"""Dump the GPU's single-graph rollouts of the C3/C5 GMM N=1000 seeds (GPU box only).

Output ``gpurun_out/batch_seqs.npz``: ``seeds`` and per seed ``s<seed>_seq`` / ``s<seed>_ranks``
/ ``s<seed>_max_rank`` for seeds 0..511 and a few of C5's seeds above 511.  The build container
picks seeds from it and certifies their sequences against the reference itself
(tests/golden/make_batch_certs.py); tests/test_gpu_batch.py then checks the batch launches'
rollouts of those seeds against the certificates.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm  # noqa: E402

N = 1000
EXTRA = [700, 1000, 1500, 2047, 3071, 4095]


def main():
    seeds = list(range(512)) + EXTRA
    eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    out = {"seeds": np.asarray(seeds, np.int32)}
    for i, s in enumerate(seeds):
        e0, e1 = gmm.gmm_pair(N, seed=s)
        eng.load_graphs([(N, e0, e1)])
        mr = int(eng.reset()[0])
        seq, ranks = eng.rollout()[0]
        out[f"s{s}_seq"] = seq.astype(np.int32)
        out[f"s{s}_ranks"] = ranks.astype(np.int32)
        out[f"s{s}_max_rank"] = np.int32(mr)
        if i % 64 == 0:
            print(f"seed {s}: {len(seq)} removals", flush=True)
    eng.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "batch_seqs.npz"), **out)
    lens = sorted(((len(out[f"s{s}_seq"]), s) for s in seeds), reverse=True)
    print("longest:", lens[:12])


if __name__ == "__main__":
    main()
