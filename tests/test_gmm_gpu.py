"""GPU Geometric Multiplex Model generator (md_gmm.hip, gmm_gpu.py).

CPU: the host pieces -- pair-index mapping, the re-decision of flagged pairs, the per-node
half of the reference generator.  GPU: exact mode equals the reference's streams graph for
graph (gmm.gmm_pair, itself pinned to the reference's golden graphs by test_gmm.py); the
device's per-node functions (Lambert W, erfinv, pow chains) against the reference's on the
same uniforms; device mode (Philox streams) is deterministic, lexicographic, and has the
reference model's edge statistics."""
import numpy as np
import pytest

from mdcommunity_amd import gmm, gmm_gpu


def test_pair_index_mapping():
    for n in (2, 3, 17, 200):
        iu, ju = np.triu_indices(n, k=1)
        i, j = gmm_gpu._pair_ij(n, np.arange(len(iu), dtype=np.int64))
        assert np.array_equal(i, iu) and np.array_equal(j, ju)


def test_redecide_matches_reference_expression():
    n = 300
    kb1, kb2, k1, k2, t1, t2, rng = gmm.node_values(n, 5)
    u = rng.random_sample(n * (n - 1) // 2)
    ref = gmm._links(k1, t1, gmm.TEMP, kb1, u)
    # a device answer with some pairs wrong, all of them flagged: the re-decision repairs it
    iu, ju = np.triu_indices(n, k=1)
    key = set((ref[:, 0].astype(np.int64) * n + ref[:, 1]).tolist())
    flag = np.array(sorted(np.random.default_rng(0).choice(len(iu), 400, replace=False)))
    flag = np.union1d(flag, np.flatnonzero(np.isin(iu * n + ju, list(key)))[:50])
    wrong = set(key)
    for p in flag[::3]:
        k = int(iu[p] * n + ju[p])
        wrong.symmetric_difference_update({k})
    w = np.array(sorted(wrong), np.int64)
    e = np.stack([w // n, w % n], axis=1).astype(np.int32)
    fixed, flips = gmm_gpu._redecide(n, e, flag.astype(np.int64), k1, t1, kb1, u)
    assert flips == len(flag[::3])
    assert np.array_equal(fixed, ref)


def test_node_values_are_gmm_pairs_first_half():
    kb1, kb2, k1, k2, t1, t2, rng = gmm.node_values(200, 7)
    npairs = 200 * 199 // 2
    e0 = gmm._links(k1, t1, gmm.TEMP, kb1, rng.random_sample(npairs))
    e1 = gmm._links(k2, t2, gmm.TEMP, kb2, rng.random_sample(npairs))
    r0, r1 = gmm.gmm_pair(200, seed=7)
    assert np.array_equal(e0, r0) and np.array_equal(e1, r1)


@pytest.mark.gpu
def test_exact_mode_equals_reference_streams():
    st = {}
    seeds = list(range(48)) + [1000, 4095]
    got = gmm_gpu.gmm_pairs(1000, seeds, exact=True, stats=st)
    for s, (e0, e1) in zip(seeds, got):
        r0, r1 = gmm.gmm_pair(1000, seed=s)
        assert np.array_equal(e0, r0) and np.array_equal(e1, r1), s
    assert st["flipped_pairs"] <= st["ambiguous_pairs"]


@pytest.mark.gpu
def test_device_node_functions_match_reference():
    rng = np.random.default_rng(3)
    G, n = 8, 1000
    u = rng.random((4, G, n))
    kbar = rng.uniform(2.0, 10.0, size=(G, 2))
    kappa, theta = gmm_gpu.node_values_device(n, u, kbar)
    for g in range(G):
        kmin1, kmin2 = gmm._kmin(kbar[g, 0], gmm.GAMMA), gmm._kmin(kbar[g, 1], gmm.GAMMA)
        k1 = kmin1 * np.power(1.0 - u[0, g], 1.0 / (1.0 - gmm.GAMMA))
        k2 = gmm._conditional_kappa(k1, u[1, g], kmin1, gmm.GAMMA, kmin2, gmm.GAMMA)
        t1 = 2.0 * np.pi * u[2, g]
        t2 = gmm._conditional_theta(t1, u[3, g], n)
        np.testing.assert_allclose(kappa[g, 0], k1, rtol=1e-13)
        np.testing.assert_allclose(kappa[g, 1], k2, rtol=1e-9)
        np.testing.assert_allclose(theta[g, 0], t1, rtol=1e-15)
        d = np.abs(theta[g, 1] - t2)
        assert np.all(np.minimum(d, 2 * np.pi - d) < 1e-9)


@pytest.mark.gpu
def test_device_mode_deterministic_and_reference_statistics():
    seeds = list(range(64))
    a = gmm_gpu.gmm_pairs(1000, seeds, exact=False)
    b = gmm_gpu.gmm_pairs(1000, seeds[:8], exact=False)
    for (x0, x1), (y0, y1) in zip(a[:8], b):
        assert np.array_equal(x0, y0) and np.array_equal(x1, y1)
    for e0, e1 in a:
        for e in (e0, e1):
            assert np.all(e[:, 0] < e[:, 1])
            k = e[:, 0].astype(np.int64) * 1000 + e[:, 1]
            assert np.all(np.diff(k) > 0)  # lexicographic, no duplicates
    ref = [gmm.gmm_pair(1000, seed=s) for s in range(64)]
    dev_m = np.array([[len(e0), len(e1)] for e0, e1 in a], float)
    ref_m = np.array([[len(e0), len(e1)] for e0, e1 in ref], float)
    # mean edges per layer over 64 graphs: kbar ~ U(2, 10) makes the per-graph count vary by
    # ~40 %, so the means of two independent samples agree within ~3 standard errors
    se = np.sqrt(dev_m.var(0) / 64 + ref_m.var(0) / 64)
    assert np.all(np.abs(dev_m.mean(0) - ref_m.mean(0)) < 3.5 * se), (dev_m.mean(0), ref_m.mean(0), se)
    # heavy-tailed degrees in both (gamma = 2.5): the largest degree well above the mean
    def dmax(e):
        return np.bincount(e.ravel(), minlength=1000).max()
    assert np.median([dmax(e0) for e0, _ in a]) > 4 * np.median(dev_m[:, 0]) * 2 / 1000
