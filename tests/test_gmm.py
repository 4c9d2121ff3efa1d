"""The vectorised GMM generator reproduces the reference generator's graphs (golden edges
were produced by U/GMM.py with random.seed(s); np.random.seed(s))."""
import numpy as np
import pytest

from conftest import load_golden
from mdcommunity_amd import gmm


@pytest.mark.parametrize("name,n,seed", [("gmm200_s7", 200, 7), ("gmm1000_s0", 1000, 0),
                                         ("gmm1000_s1", 1000, 1), ("gmm1000_s2", 1000, 2)])
def test_gmm_matches_reference(name, n, seed):
    z = load_golden(name)
    e0, e1 = gmm.gmm_pair(n, seed=seed)
    assert np.array_equal(e0, z["edges0"])
    assert np.array_equal(e1, z["edges1"])


def test_er_matches_reference():
    z = load_golden("er100")
    e0, e1 = gmm.er_pair(100, 1, 2)
    assert np.array_equal(e0, z["edges0"]) and np.array_equal(e1, z["edges1"])


def test_synthetic_dataset_graphs():
    """testSynthetic inputs (adj{1,2}_i.npy) were GMM graphs with seeds 500 + 1000 N + i."""
    import os
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "synthetic_data_g.npz"))
    for n in (32, 64):
        for i in (0, 7, 19):
            e0, e1 = gmm.gmm_pair(n, seed=500 + 1000 * n + i)
            assert np.array_equal(e0, z[f"n{n}_g{i}_e0"]) and np.array_equal(e1, z[f"n{n}_g{i}_e1"])
