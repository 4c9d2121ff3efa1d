"""Whole-sequence certificates (CPU): the GPU's removal sequence of every golden fixture,
with the REFERENCE's own Q rows, LMCC trace and AUDC along that sequence
(tests/golden/make_certificates.py runs the reference teacher-forced along it).

What is certified for each fixture:
* the GPU sequence equals the reference's up to a pinned step `prefix` (the first step where
  the GPU picks differently; only ever at a reference exact tie or a gap of a few fp32 ulps);
* from there on every GPU pick lies in the reference's own near-tie set at that state:
  max(q_ref) - q_ref[pick] <= CERT_MARGIN (the GPU's measured |dQ| at that state is checked
  on the GPU in tests/test_gpu_parity.py, which also pins the live sequence to this one);
* the reference's LMCC after every GPU removal equals the GPU's, and the reference's AUDC of
  the GPU sequence equals the reference's AUDC of its own sequence (bit-exact float64);
* the oracle, forced along the GPU sequence, reproduces the reference's rows (small fixtures).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from mdcommunity_amd import engine
from oracle import refenv, refmodel

# first step where the GPU's pick differs from the reference's (len(seq) = identical)
PINNED_PREFIX = {"er100": 19, "gmm200_s7": 7, "er300_dense": 126, "gmm1000_s0": 70, "gmm1000_s1": 23,
                 "gmm1000_s2": 55, "er1000": 163, "deg_er100": 20, "deg_gmm200_s7": 21, "deg_gmm1000_s0": 47}
CERT_MARGIN = 1e-6   # reference near-tie set: within the GPU's |dQ| bound (measured <= 1.03e-6)


def load_cert(name):
    with np.load(os.path.join(GOLDEN, f"cert_{name}.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", sorted(PINNED_PREFIX))
def test_certificate(name):
    z, c = load_golden(name), load_cert(name)
    seq, ref = c["gpu_seq"], z["seq"]
    k = int(c["prefix"])
    assert k == PINNED_PREFIX[name]
    assert seq[:k].tolist() == ref[:k].tolist()
    if k < len(ref):
        assert seq[k] != ref[k]
        # the reference itself was ambiguous at the divergence step: exact tie or a few-ulp gap
        assert z["step_stats"][k, 3] > 1 or z["step_gap"][k] < 1.2e-7
    q = c["ref_q_along"].astype(np.float64)
    assert q.shape == (len(seq), int(z["n_nodes"]))
    margin = np.array([np.nanmax(q[t]) - q[t][seq[t]] for t in range(len(seq))])
    assert np.array_equal(margin, c["margin"])
    assert margin.min() >= 0.0 and margin.max() <= CERT_MARGIN, margin.max()
    assert np.all(margin[:k] == 0.0)
    # the reference's rows along its own trajectory equal the forced rows on the common prefix
    qr = z["q_rows"][:k]
    qa = np.where(np.isnan(q[:k]), -(2147483647 / 2), q[:k])
    assert np.array_equal(qr, qa)
    # LMCC trace and AUDC along the GPU sequence (reference env), AUDC = the golden's
    assert float(c["ref_score_along"]) == float(z["score"])
    assert int(c["ref_ranks_along"][-1]) == int(z["ranks"][-1])


def test_certificate_meta_consistent():
    meta = json.load(open(os.path.join(GOLDEN, "meta_certificates.json")))
    for name, k in PINNED_PREFIX.items():
        assert meta[name]["prefix"] == k and meta[name]["audc_equal"]


@pytest.mark.parametrize("name", ["er100", "gmm200_s7", "deg_gmm200_s7"])
def test_oracle_along_gpu_sequence(name):
    """The oracle forced along the GPU's sequence gives the reference's certificate rows
    (bit-identical on the build host; 1e-6 elsewhere) and LMCC trace."""
    import torch
    torch.set_num_threads(16)
    z, c = load_golden(name), load_cert(name)
    cost = "degree" if name.startswith("deg_") else "unit"
    w = refmodel.RefWeights.load(engine.DEFAULT_DEGREE if cost == "degree" else engine.DEFAULT_UNIT)
    g = refenv.RefGraph(int(z["n_nodes"]), z["edges0"], z["edges1"])
    env = refenv.RefEnv(g, cost)
    ranks = []
    for t, a in enumerate(c["gpu_seq"]):
        assert not env.terminal()
        q = refenv.predict(w, g, env.covered, env.removed, cost)
        ref = c["ref_q_along"][t].astype(np.float64)
        live = ~np.isnan(ref)
        assert np.array_equal(q != refenv.MASK, live)
        assert np.max(np.abs(q[live] - ref[live])) <= 1e-6
        ranks.append(env.step(int(a)))
    assert env.terminal()
    assert ranks == c["ref_ranks_along"].tolist()
    assert env.score == float(c["ref_score_along"])
