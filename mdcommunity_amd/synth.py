"""Synthetic stand-in for the reference's testReal inputs (BASELINE.json configs[3]).

The reference's real multiplex files (``data/real/*.edges``) are not in the repository; its
committed results show what they look like: homo_genetic_multiplex has N = 18 222 nodes and
the unit-cost rollout needed 2 081 removals (``results/unitcost/MultiDismantler_real/
StepRatio_0.0000/``).  ``real_like_multiplex`` writes a file of that shape in the same
``layer u v`` format (1-based ids, read by ``MultiDismantler.read_multiplex``): two sparse
layers on the same node ids with heavy-tailed (Chung-Lu, power-law) degrees, hubs partly
shared between the layers, many nodes absent from a layer (degree 0), duplicate edges and a
few self-loops (both dropped by the reader, as the reference's reader does).  Deterministic
per seed (numpy RandomState).
"""
import numpy as np


def real_like_layers(n=18000, seed=0, mean_deg=3.0, gamma=2.3, shared=0.6):
    """Two edge lists [(u, v)] (0-based, file order, duplicates/self-loops included)."""
    rs = np.random.RandomState(seed)
    # Chung-Lu weights w_i ~ i^(-1/(gamma-1)) over a random node order per layer; a fraction
    # `shared` of the nodes keeps its rank in both layers (hubs in common)
    rank = np.arange(1, n + 1, dtype=np.float64)
    w = rank ** (-1.0 / (gamma - 1.0))
    order0 = rs.permutation(n)
    order1 = order0.copy()
    move = rs.rand(n) >= shared
    idx = np.flatnonzero(move)
    order1[idx] = order0[rs.permutation(idx)]
    layers = []
    for order in (order0, order1):
        p = np.empty(n)
        p[order] = w
        p /= p.sum()
        m = int(mean_deg * n / 2)
        u = rs.choice(n, size=m, p=p)
        v = rs.choice(n, size=m, p=p)
        layers.append(list(zip(u.tolist(), v.tolist())))
    return layers


def write_real_like(path, n=18000, seed=0, **kw):
    """Writes the ``layer u v`` file; returns (n, edges per layer as written)."""
    layers = real_like_layers(n, seed, **kw)
    with open(path, "w") as f:
        for lid, edges in enumerate(layers, start=1):
            for u, v in edges:
                f.write("%d %d %d\n" % (lid, u + 1, v + 1))
    return n, [len(e) for e in layers]
