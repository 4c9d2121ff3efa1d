"""Geometric Multiplex Model generator on the GPU (md_gmm.hip).

The reference draws its synthetic two-layer graphs with U/GMM.py:6-68 (U/Hyperbolic.py:18-117):
per node kappa / theta of two layers, then one uniform per node pair per layer -- an O(N^2)
Python loop (~4 s per N = 1000 graph there, ~45 ms for the vectorised host restatement
``gmm.gmm_pair``).  Here the pair loop runs on the device, one workgroup per layer, and writes
the edges in the reference's lexicographic order.

* ``gmm_pairs(n, seeds, exact=True)``: the reference's own streams -- kbar from Python's
  ``random``, the per-node values and the pair uniforms from numpy's legacy stream, drawn on
  the host exactly as ``gmm.gmm_pair`` draws them; the device evaluates the link test, and
  every pair it flags as within a relative 1e-9 of the threshold is re-decided here with the
  reference's expression (``gmm.link_keep``), so the graphs equal ``gmm.gmm_pair``'s.
* ``gmm_pairs(n, seeds, exact=False)``: everything on the device -- Philox4x32-10 streams keyed
  by the seed, the per-node values computed there (Lambert W by Halley steps, erfinv).  The
  same model, not the numpy stream (so the committed fixtures stay the parity source, as
  SURVEY.md §8(f3) says); deterministic per seed.
"""
import ctypes

import numpy as np

from . import _lib, gmm

TEMP = gmm.TEMP
_u64p = ctypes.POINTER(ctypes.c_uint64)


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _check(st):
    if st != _lib.MD_OK:
        raise _lib.MDError(f"{_lib.STATUS_NAMES.get(st, st)}: {_lib.load_library().md_gmm_last_error().decode()}")


def _pair_ij(n, p):
    """Row-major pair index (i < j) -> (i, j)."""
    i_all = np.arange(n - 1, dtype=np.int64)
    starts = i_all * (n - 1) - i_all * (i_all - 1) // 2
    i = np.searchsorted(starts, p, side="right") - 1
    j = p - starts[i] + i + 1
    return i.astype(np.int64), j.astype(np.int64)


def _links(n, kappa, theta, mu, device, uniforms=None, seeds=None, edge_cap=None):
    """md_gmm_links over L = kappa.shape[0] layers: list of [E, 2] int32 edge arrays, and the
    ambiguous pair indices per layer (exact mode)."""
    lib = _lib.load_library()
    L = kappa.shape[0]
    cap = int(edge_cap or max(64 * n, 4096))
    acap = 4096
    edges = np.zeros((L, cap, 2), np.int32)
    ecnt = np.zeros(L, np.int64)
    amb = np.zeros((L, acap), np.int64)
    acnt = np.zeros(L, np.int64)
    kappa = np.ascontiguousarray(kappa, np.float64)
    theta = np.ascontiguousarray(theta, np.float64)
    mu = np.ascontiguousarray(mu, np.float64)
    un = np.ascontiguousarray(uniforms, np.float64) if uniforms is not None else None
    sd = np.ascontiguousarray(seeds, np.uint64) if seeds is not None else None
    _check(lib.md_gmm_links(int(device), L, int(n), _p(kappa, _lib._f64p), _p(theta, _lib._f64p), _p(mu, _lib._f64p),
                            _p(un, _lib._f64p), _p(sd, _u64p), _p(edges, _lib._i32p), _p(ecnt, _lib._i64p), cap,
                            _p(amb, _lib._i64p), _p(acnt, _lib._i64p), acap))
    return [edges[l, :ecnt[l]].copy() for l in range(L)], [amb[l, :acnt[l]].copy() for l in range(L)]


def _redecide(n, e, amb, kappa, theta, kbar, u):
    """Edges of one layer with the ambiguous pairs decided by the reference's expression."""
    if len(amb) == 0:
        return e, 0
    i, j = _pair_ij(n, amb)
    keep = gmm.link_keep(kappa, theta, TEMP, kbar, u[amb], i, j)
    key = e[:, 0].astype(np.int64) * n + e[:, 1]
    pk = i * n + j
    have = np.isin(pk, key)
    flips = int(np.count_nonzero(have != keep))
    if flips:
        key = np.union1d(np.setdiff1d(key, pk[have & ~keep]), pk[keep & ~have])
        e = np.stack([key // n, key % n], axis=1).astype(np.int32)
    return e, flips


def gmm_pairs(n, seeds, exact=True, device=0, batch=None, stats=None):
    """Two-layer GMM graphs for each seed: list of (edges0, edges1), [E, 2] int32, u < v in
    lexicographic order.  exact=True: equal to gmm.gmm_pair(n, seed) (the reference's
    streams); exact=False: device Philox streams (same model, not the numpy stream)."""
    seeds = [int(s) for s in seeds]
    # graphs per device call: exact mode holds the pair uniforms of each graph (8 MB at N = 1000)
    batch = batch or (16 if exact else 128)
    out = []
    npairs = n * (n - 1) // 2
    flips = 0
    ambs = 0
    for b0 in range(0, len(seeds), batch):
        chunk = seeds[b0:b0 + batch]
        G = len(chunk)
        if exact:
            kappa = np.empty((2 * G, n))
            theta = np.empty((2 * G, n))
            kbar = np.empty(2 * G)
            u = np.empty((2 * G, npairs))
            for g, s in enumerate(chunk):
                kb1, kb2, k1, k2, t1, t2, rng = gmm.node_values(n, s)
                kappa[2 * g], kappa[2 * g + 1], theta[2 * g], theta[2 * g + 1] = k1, k2, t1, t2
                kbar[2 * g], kbar[2 * g + 1] = kb1, kb2
                u[2 * g] = rng.random_sample(npairs)  # layer 0's pairs, then layer 1's (GMM.py:26-27)
                u[2 * g + 1] = rng.random_sample(npairs)
            mu = gmm.link_mu(TEMP, kbar)
            es, am = _links(n, kappa, theta, mu, device, uniforms=u)
            for l in range(2 * G):
                es[l], f = _redecide(n, es[l], am[l], kappa[l], theta[l], kbar[l], u[l])
                flips += f
                ambs += len(am[l])
        else:
            sd = np.asarray(chunk, np.uint64)
            kbar = np.empty(2 * G)
            kappa = np.empty((G, 2, n))
            theta = np.empty((G, 2, n))
            lib = _lib.load_library()
            _check(lib.md_gmm_nodes(int(device), G, int(n), _p(sd, _u64p), None, None, _p(kbar, _lib._f64p),
                                    _p(kappa, _lib._f64p), _p(theta, _lib._f64p)))
            mu = gmm.link_mu(TEMP, kbar)
            es, _ = _links(n, kappa.reshape(2 * G, n), theta.reshape(2 * G, n), mu, device, seeds=sd)
        for g in range(G):
            out.append((es[2 * g], es[2 * g + 1]))
    if stats is not None:
        stats["ambiguous_pairs"] = ambs
        stats["flipped_pairs"] = flips
    return out


def node_values_device(n, uniforms, kbar, device=0):
    """The device's per-node functions on given uniforms [4][G][n] and kbar [G][2] (for checks
    against the reference's own functions): (kappa [G][2][n], theta [G][2][n])."""
    lib = _lib.load_library()
    uniforms = np.ascontiguousarray(uniforms, np.float64)
    kbar = np.ascontiguousarray(kbar, np.float64)
    G = uniforms.shape[1]
    kb = np.empty(2 * G)
    kappa = np.empty((G, 2, n))
    theta = np.empty((G, 2, n))
    _check(lib.md_gmm_nodes(int(device), G, int(n), None, _p(uniforms, _lib._f64p), _p(kbar, _lib._f64p),
                            _p(kb, _lib._f64p), _p(kappa, _lib._f64p), _p(theta, _lib._f64p)))
    return kappa, theta
