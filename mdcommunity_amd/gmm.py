"""Geometric Multiplex Model generator (synthetic two-layer test graphs).

Vectorised restatement of the reference generator ``U/GMM.py:6-68`` with the hyperbolic
helpers of ``U/Hyperbolic.py:18-117``: g = 0.5, nu = 0.2, gamma = 2.5, T = 0.4,
kbar_l ~ U(2, 10).  It draws from the same two random streams in the same order as the
reference (Python ``random`` for kbar, numpy's legacy global stream for everything else:
N kappa, N conditional kappa, N theta, N conditional theta, then one draw per node pair
(i < j) per layer), so a given seed reproduces the reference's graph exactly
(``tests/test_gmm.py`` checks the golden N=200/1000 graphs).  The O(N^2) pair loop of
``CreateNetworks`` is one array expression here.
"""
import random as _pyrandom

import numpy as np
from scipy.special import erf, erfinv, lambertw

NU = 0.2
G_CORR = 0.5
GAMMA = 2.5
TEMP = 0.4


def _kmin(kbar, gamma):
    return kbar * (gamma - 2.0) / (gamma - 1)


def _conditional_kappa(kappa1, u, kmin1, gamma1, kmin2, gamma2, nu=NU):
    phi = -np.log(1.0 - np.power((kmin1 / kappa1), (gamma1 - 1.0)))
    z = 1.0 / kmin1 * np.power(phi, (nu / (nu - 1.0))) * np.power(kappa1, -gamma1)
    z = z * (kmin1 * np.power(kappa1, gamma1) - np.power(kmin1, gamma1) * kappa1)
    zr = z * u
    zr = (nu / (1.0 - nu)) * lambertw(np.power(zr, ((nu - 1.0) / nu)) / (nu / (1.0 - nu)))
    zr = np.power(zr, (1.0 / (1.0 - nu))) - np.power(phi, (1.0 / (1.0 - nu)))
    zr = np.exp(-np.power(zr, (1.0 - nu)))
    zr = kmin2 * np.power(1.0 - zr, (1.0 / (1.0 - gamma2)))
    return np.asarray(zr).real


def _conditional_theta(theta1, u, n, g=G_CORR):
    two_pi = 2 * np.pi
    sigma0 = n / (4.0 * np.pi)
    if sigma0 > 100.0:
        sigma0 = 100.0
    sigma = sigma0 * (1.0 / g - 1.0)
    ell = np.sqrt(2.0) * sigma * erfinv((-1.0 + 2.0 * u) * erf(n / (2 * np.sqrt(2) * sigma)))
    return np.mod(theta1 + two_pi * ell / n, two_pi)


def link_mu(temp, kbar):
    """CreateNetworks' mu (U/Hyperbolic.py:101-117)."""
    return np.sin(temp * np.pi) / (2 * np.pi * temp * kbar)


def link_keep(kappa, theta, temp, kbar, u, iu, ju):
    """The link test of CreateNetworks for the pairs (iu, ju) with their uniforms u (also used
    by gmm_gpu to re-decide the pairs the device flags as within rounding of the threshold)."""
    n = len(kappa)
    two_pi = 2 * np.pi
    dtheta = n / (two_pi) * np.abs(np.pi - np.abs(np.pi - np.abs(theta[iu] - theta[ju])))
    mu = link_mu(temp, kbar)
    r = dtheta / (mu * kappa[iu] * kappa[ju])
    return u < (1.0 / (1.0 + np.power(r, 1.0 / temp)))


def _links(kappa, theta, temp, kbar, u):
    """CreateNetworks (U/Hyperbolic.py:101-117): pairs (i<j) in row-major order."""
    n = len(kappa)
    iu, ju = np.triu_indices(n, k=1)
    keep = link_keep(kappa, theta, temp, kbar, u, iu, ju)
    return np.stack([iu[keep], ju[keep]], axis=1).astype(np.int32)


def node_values(n, seed=None, py_rng=None, np_rng=None):
    """The per-node half of gmm_pair: (kbar1, kbar2, kappa1, kappa2, theta1, theta2, np_rng),
    the numpy stream left where the pair draws start (U/GMM.py:10-25)."""
    if seed is not None:
        py_rng = _pyrandom.Random(seed)
        np_rng = np.random.RandomState(seed)
    kbar1 = py_rng.uniform(2.0, 10.0)
    kbar2 = py_rng.uniform(2.0, 10.0)
    kmin1, kmin2 = _kmin(kbar1, GAMMA), _kmin(kbar2, GAMMA)
    kappa1 = kmin1 * np.power(1.0 - np_rng.random_sample(n), 1.0 / (1.0 - GAMMA))
    kappa2 = _conditional_kappa(kappa1, np_rng.random_sample(n), kmin1, GAMMA, kmin2, GAMMA)
    theta1 = 2.0 * np.pi * np_rng.random_sample(n)
    theta2 = _conditional_theta(theta1, np_rng.random_sample(n), n)
    return kbar1, kbar2, kappa1, kappa2, theta1, theta2, np_rng


def gmm_pair(n, seed=None, py_rng=None, np_rng=None):
    """Two-layer GMM graph on n nodes: returns (edges0, edges1), each [E, 2] int32 with u < v
    in lexicographic order (the networkx ``G.edges()`` order of the reference's graphs).

    With ``seed`` the streams are ``random.seed(seed); np.random.seed(seed)`` as the
    reference's callers do; otherwise pass ``random.Random`` / ``RandomState`` instances."""
    kbar1, kbar2, kappa1, kappa2, theta1, theta2, np_rng = node_values(n, seed, py_rng, np_rng)
    npairs = n * (n - 1) // 2
    e0 = _links(kappa1, theta1, TEMP, kbar1, np_rng.random_sample(npairs))
    e1 = _links(kappa2, theta2, TEMP, kbar2, np_rng.random_sample(npairs))
    return e0, e1


def er_pair(n, seed1, seed2, p=None):
    """Two independent Erdos-Renyi layers as networkx.erdos_renyi_graph(n, p, seed) -> edge
    lists in from_numpy_array order (the SURVEY's ER control graphs)."""
    import networkx as nx
    p = 4.0 / n if p is None else p
    out = []
    for s in (seed1, seed2):
        a = nx.to_numpy_array(nx.erdos_renyi_graph(n, p, seed=s))
        out.append(np.argwhere(np.triu(a) > 0).astype(np.int32))
    return out[0], out[1]
