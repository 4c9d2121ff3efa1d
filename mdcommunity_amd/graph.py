"""Graph containers of the rollout (drop-in for ``U/graph.py``).

``Graph_test(G1, G2)`` (``U/graph.py:69-84``) keeps the reference's attributes
(``num_nodes``, ``adj_list``, ``edge_list``, ``num_edges``, ``max_rank``, ``weights``) and
adds the flat edge arrays the device engine consumes (``edges[l]``: [E_l, 2] int32 in
networkx ``G.edges()`` order, which fixes the neighbour-aggregation order).
``max_rank`` (the initial mutual-LMCC size, ``U/graph.py:80-84``) is computed by the
device MCC kernel (``md_reset``) the first time it is needed.

``Graph(N)`` (``U/graph.py:7-30``) draws a GMM multiplex with :mod:`mdcommunity_amd.gmm`;
``GSet`` is the graph pool of ``U/graph.py:49-67``.
"""
import random as _pyrandom

import numpy as np

from . import gmm


class _EdgeSet:
    """Graph_test from raw edge arrays (no networkx needed)."""

    def _init_edges(self, n, edges0, edges1, weights=None):
        self.num_nodes = int(n)
        self.edges = [np.ascontiguousarray(np.asarray(e, dtype=np.int32).reshape(-1, 2)) for e in (edges0, edges1)]
        self.edge_list = [[(int(u), int(v)) for u, v in e] for e in self.edges]
        self.num_edges = [len(self.edges[0]), len(self.edges[1])]
        self.adj_list = []
        for l in range(2):
            nb = [[] for _ in range(self.num_nodes)]
            for u, v in self.edges[l]:
                nb[u].append(int(v))
                nb[v].append(int(u))
            self.adj_list.append(list(enumerate(nb)))
        self.weights = weights if weights is not None else [{}, {}]
        self._max_rank = None

    @property
    def max_rank(self):
        if self._max_rank is None:
            from .engine import initial_lmcc
            self._max_rank = int(initial_lmcc(self))
        return self._max_rank

    @max_rank.setter
    def max_rank(self, v):
        self._max_rank = int(v)


class Graph_test(_EdgeSet):  # noqa: N801 (reference name)
    """Two networkx layers on the same node ids 0..N-1 (U/graph.py:69-84)."""

    def __init__(self, G1=None, G2=None, *, edges=None, n=None, weights=None):
        if edges is not None:
            self._init_edges(n, edges[0], edges[1], weights)
            return
        n = len(G1.nodes)
        e = []
        for g in (G1, G2):
            lst = [(int(u), int(v)) for u, v in g.edges()]
            e.append(np.asarray(lst, dtype=np.int32).reshape(-1, 2))
        self._init_edges(n, e[0], e[1], weights)

    @classmethod
    def from_edges(cls, n, edges0, edges1, weights=None):
        return cls(edges=(edges0, edges1), n=n, weights=weights)


class Graph(_EdgeSet):
    """GMM random multiplex on N nodes (U/graph.py:7-30); Graph(0) is an empty placeholder."""

    def __init__(self, N=0, seed=None):
        if N == 0:
            self.num_nodes = 0
            self.edges = [np.zeros((0, 2), np.int32), np.zeros((0, 2), np.int32)]
            self.edge_list = [[], []]
            self.num_edges = []
            self.adj_list = []
            self.weights = [{}, {}]
            self._max_rank = 0
            return
        if seed is None:
            e0, e1 = gmm.gmm_pair(N, py_rng=_pyrandom, np_rng=np.random.mtrand._rand)
        else:
            e0, e1 = gmm.gmm_pair(N, seed=seed)
        self._init_edges(N, e0, e1)


class GSet:
    """Graph pool keyed by integer id (U/graph.py:49-67)."""

    def __init__(self):
        self.graph_pool = {}

    def InsertGraph(self, gid, graph):  # noqa: N802
        assert gid not in self.graph_pool
        self.graph_pool[gid] = graph

    def Sample(self):  # noqa: N802
        assert self.graph_pool
        gid = np.random.choice(list(self.graph_pool.keys()))
        return self.graph_pool[gid]

    def Get(self, gid):  # noqa: N802
        assert gid in self.graph_pool
        return self.graph_pool[gid]

    def Clear(self):  # noqa: N802
        self.graph_pool.clear()


def ensure_degree_weights(g):
    """Graph_test.weights of the degree-cost variant (D/graph.py:80-115): filled when the
    initial LMCC is not 1, as w_l[v] = deg_l(v) / maxdeg_l on the original layers (Python
    int / int division, node order 0..N-1)."""
    if g.weights[0] or g.max_rank == 1:
        return g.weights
    for l in range(2):
        d = np.bincount(g.edges[l].reshape(-1), minlength=g.num_nodes)
        mx = int(d.max())
        g.weights[l] = {v: int(d[v]) / mx for v in range(g.num_nodes)}
    return g.weights


def node_weight_array(graphs):
    """Device layout of the degree-cost node inputs: float32 [2][sum N] (layer-major)."""
    out = []
    for l in range(2):
        parts = []
        for g in graphs:
            w = ensure_degree_weights(g)[l]
            parts.append(np.asarray([w.get(v, 0.0) for v in range(g.num_nodes)], dtype=np.float64))
        out.append(np.concatenate(parts) if parts else np.zeros(0))
    return np.concatenate(out).astype(np.float32)


def degree_weights(g):
    """Degree-cost node weights w_l(v) = deg_l(v) / maxdeg_l on the original layers
    (D/graph.py:91-115); returns float64 arrays [2][N] and the python-sum totals W_l."""
    out = []
    for l in range(2):
        d = np.bincount(g.edges[l].reshape(-1), minlength=g.num_nodes).astype(np.int64)
        mx = int(d.max()) if d.size else 0
        out.append(np.array([di / mx if mx else 0.0 for di in d], dtype=np.float64))
    return out
