"""CPU checks of the batch certificates (tests/golden/batch_certs.npz, made by
tests/golden/make_batch_certs.py from the reference itself): the seeds' graphs come from the
build's generator (mdcommunity_amd.gmm = U/GMM.py's streams), and the oracle environment stepped
along each certified GPU sequence gives the reference's LMCC trace and AUDC bit for bit
(U/mvc_env.py:74-87,128-137, U/Mcc.py:30-38) and ends terminal with the last removal."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import refenv
from mdcommunity_amd import gmm

N = 1000


def certs():
    with np.load(os.path.join(GOLDEN, "batch_certs.npz")) as z:
        return {k: z[k] for k in z.files}


C = certs()


@pytest.mark.parametrize("seed", C["seeds"].tolist())
def test_batch_cert_against_oracle(seed):
    e0, e1 = gmm.gmm_pair(N, seed=seed)
    g = refenv.RefGraph(N, e0, e1)
    assert g.max_rank == int(C[f"s{seed}_max_rank"])
    env = refenv.RefEnv(g, "unit")
    seq = C[f"s{seed}_gpu_seq"].tolist()
    for a in seq:
        assert not env.terminal()
        env.step(int(a))
    assert env.terminal()
    assert env.ranks == C[f"s{seed}_ref_ranks_along"].tolist()
    assert env.score == float(C[f"s{seed}_ref_score_along"]) == float(C[f"s{seed}_ref_score"])
    # the GPU's sequence agrees with the reference's own up to a tie / near-tie of the reference
    ref = C[f"s{seed}_ref_seq"].tolist()
    assert len(ref) == len(seq)
    assert float(np.max(C[f"s{seed}_margin"])) <= 2e-5
