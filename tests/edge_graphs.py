"""The synthetic edge-case graphs of tests/test_gpu_edge_cases.py (seeded), shared with the
generator of their reference goldens (tests/golden/make_golden_edge.py).  Pure numpy: no GPU,
no reference import."""
import numpy as np


def er_edges(rng, nodes, p):
    nodes = np.asarray(nodes)
    out = []
    for i in range(len(nodes)):
        for j in range(i + 1, len(nodes)):
            if rng.random() < p:
                out.append((int(nodes[i]), int(nodes[j])))
    rng.shuffle(out)
    return np.array(out, np.int32).reshape(-1, 2)


def cases():
    rng = np.random.default_rng(2026)
    star = np.array([(0, v) for v in range(1, 100)], np.int32)
    tree = np.array([(int(rng.integers(0, v)), v) for v in range(1, 130)], np.int32)
    c1, c2 = np.arange(0, 100), np.arange(100, 200)
    return [
        ("k2", 2, np.array([[0, 1]], np.int32), np.array([[0, 1]], np.int32)),
        ("path_triangle", 3, np.array([[0, 1], [1, 2]], np.int32), np.array([[0, 1], [1, 2], [0, 2]], np.int32)),
        ("shared_hub_star", 100, star, star[::-1].copy()),
        ("isolated_nodes", 50, er_edges(rng, range(40), 0.15), er_edges(rng, range(40), 0.12)),
        ("wave_63", 63, er_edges(rng, range(63), 0.08), er_edges(rng, range(63), 0.1)),
        ("wave_65", 65, er_edges(rng, range(65), 0.08), er_edges(rng, range(65), 0.1)),
        ("two_clusters", 200, np.concatenate([er_edges(rng, c1, 0.06), er_edges(rng, c2, 0.05)]),
         np.concatenate([er_edges(rng, c1, 0.05), er_edges(rng, c2, 0.07)])),
        ("tree_vs_dense", 130, tree, er_edges(rng, range(130), 0.2)),
        ("layer1_empty", 20, er_edges(rng, range(20), 0.3), np.zeros((0, 2), np.int32)),
    ]
