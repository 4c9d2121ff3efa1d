"""The confirmation shortcut of the device's mutual-LMCC fixed point (md_env.h mcc_fixed_point,
MD_FP_SHORTCUT) restated on the CPU and checked against the reference's alternating fixed point
(oracle.refenv.mutual_components, U/Mcc.py:30-38) on random two-layer graphs.

The device runs Jacobi rounds: union both layers (recording the edges that linked two trees, a
spanning forest F_l), label, and while the partitions differ prune every edge crossing the
other layer's partition.  The shortcut ends the fixed point after a prune when
#C_l + (pruned edges of F_l) == #classes of C0 ^ C1 for both layers.  The claim is that the
partition, the pruned-edge set and hence the LMCC are then exactly those of running the rounds
to the end -- for any union order (the device's is concurrent), so the union order is shuffled
here.  CPU only: the device path is covered by the GPU suites (identical rollouts with the
switch on and off)."""
import random

import networkx as nx

from oracle import refenv


def _find(par, x):
    while par[x] != x:
        par[x] = par[par[x]]
        x = par[x]
    return x


def device_fixed_point(n, edges, cover, shortcut, rng):
    """edges: list of (layer, u, v) alive edges.  Returns (labels of the final partition as a
    frozenset of frozensets, pruned edge set, rounds)."""
    alive = [e for e in edges if e[1] != cover and e[2] != cover]
    pruned = set()
    rounds = 0
    while True:
        rounds += 1
        par = [list(range(n)), list(range(n))]
        tree = [False] * len(alive)
        order = list(range(len(alive)))
        rng.shuffle(order)
        for i in order:
            l, u, v = alive[i]
            a, b = _find(par[l], u), _find(par[l], v)
            if a != b:
                if a > b:
                    a, b = b, a
                par[l][b] = a  # link the larger root under the smaller (min-id roots)
                tree[i] = True
        lab = [[_find(par[l], x) for x in range(n)] for l in range(2)]
        if lab[0] == lab[1]:
            part = lab[0]
            break
        nc = [sum(1 for x in range(n) if lab[l][x] == x) for l in range(2)]
        keep, t = [], [0, 0]
        for i, (l, u, v) in enumerate(alive):
            other = lab[1 - l]
            if other[u] != other[v]:
                pruned.add((l, u, v))
                t[l] += tree[i]
            else:
                keep.append((l, u, v))
        alive = keep
        pairs = list(zip(lab[0], lab[1]))
        npart = len(set(pairs))
        if shortcut and nc[0] + t[0] == npart and nc[1] + t[1] == npart:
            part = pairs
            break
    classes = {}
    for x in range(n):
        classes.setdefault(part[x], set()).add(x)
    return frozenset(frozenset(c) for c in classes.values()), pruned, rounds


def reference_fixed_point(n, edges, cover):
    g = [nx.Graph(), nx.Graph()]
    for l in range(2):
        g[l].add_nodes_from(x for x in range(n) if x != cover)
    for l, u, v in edges:
        if u != cover and v != cover:
            g[l].add_edge(u, v)
    removed = [set(), set()]
    comps = refenv.mutual_components(g[0], g[1], removed)
    part = frozenset(frozenset(c) for c in comps) | {frozenset([cover])}
    pruned = {(l, u, v) for l, u, v in edges if (u, v) in removed[l] or (v, u) in removed[l]}
    return part, pruned


def random_multiplex(n, p0, p1, seed):
    rng = random.Random(seed)
    edges = []
    for l, p in enumerate((p0, p1)):
        for u in range(n):
            for v in range(u + 1, n):
                if rng.random() < p:
                    edges.append((l, u, v))
    return edges


def test_shortcut_equals_full_rounds_and_reference():
    saved = total = 0
    for seed in range(40):
        n = 40 + seed % 3 * 20
        edges = random_multiplex(n, 2.2 / n, 2.6 / n, seed)
        rng = random.Random(1000 + seed)
        for cover in rng.sample(range(n), 4):
            full = device_fixed_point(n, edges, cover, False, random.Random(seed * 7 + cover))
            short = device_fixed_point(n, edges, cover, True, random.Random(seed * 7 + cover))
            ref_part, ref_pruned = reference_fixed_point(n, edges, cover)
            assert full[0] == ref_part and full[1] == ref_pruned
            assert short[0] == ref_part and short[1] == ref_pruned, (seed, cover)
            total += full[2]
            saved += full[2] - short[2]
    assert saved > 0  # the shortcut does end fixed points early on these graphs
    assert saved < total


def test_shortcut_over_a_rollout_prefix():
    """Successive removals on one graph (the state carries the pruned edges forward, as a
    rollout does): the shortcut's partition and pruned set equal the reference's at every step."""
    n = 120
    edges = random_multiplex(n, 2.8 / n, 3.0 / n, 7)
    rng = random.Random(3)
    alive = list(edges)
    covered = set()
    for step in range(25):
        live = sorted({u for _, u, v in alive} | {v for _, u, v in alive})
        if not live:
            break
        a = rng.choice(live)
        part_s, pruned_s, _ = device_fixed_point(n, alive, a, True, random.Random(step))
        part_r, pruned_r = reference_fixed_point(n, alive, a)
        for c in covered:  # covered nodes are singletons in both
            part_r = part_r | {frozenset([c])}
        assert {c for c in part_s if len(c) > 1} == {c for c in part_r if len(c) > 1}
        assert pruned_s == pruned_r
        covered.add(a)
        alive = [e for e in alive if e not in pruned_s and a not in (e[1], e[2])]
