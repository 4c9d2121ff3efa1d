"""The batched-prefix environment step (md_env.h team_prefix_step) rests on one property of the
reference's mutual-LMCC cascade (U/Mcc.py:30-38, U/mvc_env.py:74-87,140-162):

    the state after covering a_1..a_j one by one from a fixed-point state S (a cascade after
    each cover) has the same alive edges, LMCC and partition as ONE cascade of S with all of
    a_1..a_j covered at once.

(The fixed point is the coarsest partition whose classes are connected in both layers by edges
inside them; a valid partition of G - S_j is valid for G - S_(j-1), so the partitions only get
finer, and an edge pruned earlier crosses every later partition.)  The reference's bookkeeping
splits the dead edges into covered ones (numCoveredEdges: alive when an endpoint was covered) and
pruned ones (remove_edge); with d(e) = the first prefix whose state lacks edge e, e is covered iff
it touches a_d(e).  The picks stop at the first terminal state (GetSolution's `continue`,
U/MultiDismantler_torch.py:725-735).

This CPU test checks that property with the oracle (tests only) on random graphs, random start
states and random pick lists: LMCC after every pick, covered / pruned counters, the removed-edge
sets, the alive edges and the terminal truncation all equal the sequential env's."""
import numpy as np
import pytest

from oracle import refenv
from mdcommunity_amd import gmm


def alive_edges(graph, covered, removed):
    out = set()
    for l in range(2):
        for k, (u, v) in enumerate(graph.edge_list[l]):
            if u not in covered and v not in covered and (u, v) not in removed[l]:
                out.add((l, k))
    return out


def prefix_batch(graph, covered0, removed0, picks):
    """Every prefix's state from the start state alone, then the death-step bookkeeping."""
    start = alive_edges(graph, covered0, removed0)
    states, lm = [], []
    for j in range(1, len(picks) + 1):
        cov = set(covered0) | set(picks[:j])
        rem = [set(removed0[0]), set(removed0[1])]
        g1, g2 = graph.nx_layers(cov, rem)
        lm.append(refenv.lmcc_size(refenv.mutual_components(g1, g2, rem)))
        states.append(alive_edges(graph, cov, rem))
    for j in range(1, len(states)):
        assert states[j] <= states[j - 1]  # nested
    # terminal truncation: pick j is applied iff the state after j - 1 picks is not terminal
    J = len(picks)
    for j, s in enumerate(states, 1):
        if not any(l == 0 for l, _ in s) or not any(l == 1 for l, _ in s):
            J = j
            break
    cov_cnt, pr_cnt = [0, 0], [0, 0]
    pruned = [set(), set()]
    for (l, k) in start:
        d = next((j for j in range(1, J + 1) if (l, k) not in states[j - 1]), None)
        if d is None:
            continue
        u, v = graph.edge_list[l][k]
        if picks[d - 1] in (u, v):
            cov_cnt[l] += 1
        else:
            pr_cnt[l] += 1
            pruned[l] |= {(u, v), (v, u)}
    return J, lm[:J], cov_cnt, pr_cnt, pruned, states[J - 1] if J else start


def er_graph(n, p, rng):
    iu = np.triu_indices(n, 1)
    out = []
    for _ in range(2):
        m = rng.random(len(iu[0])) < p
        out.append(np.stack([iu[0][m], iu[1][m]], 1).astype(np.int32))
    return out


CASES = [("er", 60, 0.08, s) for s in range(6)] + [("gmm", 150, None, s) for s in range(4)]


@pytest.mark.parametrize("kind,n,p,seed", CASES)
def test_prefix_states_equal_sequential(kind, n, p, seed):
    rng = np.random.default_rng(100 + seed)
    if kind == "er":
        e0, e1 = er_graph(n, p, rng)
    else:
        e0, e1 = gmm.gmm_pair(n, seed=seed)
    g = refenv.RefGraph(n, e0, e1)
    env = refenv.RefEnv(g, "unit")
    # a random start state: a few sequential steps
    for _ in range(int(rng.integers(0, 4))):
        live = refenv.featurize(g, env.covered, env.removed)[0]
        if not live or env.terminal():
            break
        env.step(int(rng.choice(live)))
    if env.terminal():
        return
    cov0 = set(env.covered)
    rem0 = [set(env.removed[0]), set(env.removed[1])]
    nc0 = list(env.num_covered)
    # picks: live nodes mostly, some isolated non-covered nodes too, no repeats
    free = [v for v in range(n) if v not in cov0]
    k = int(rng.integers(2, min(len(free), 40)))
    picks = [int(x) for x in rng.choice(free, size=k, replace=False)]
    J, lm, cc, pc, pruned, final = prefix_batch(g, cov0, rem0, picks)
    # sequential (the reference's loop)
    seq_lm = []
    for a in picks:
        if env.terminal():
            break
        seq_lm.append(env.step(a))
    assert len(seq_lm) == J
    assert seq_lm == lm
    assert env.num_covered == [nc0[0] + cc[0], nc0[1] + cc[1]]
    for l in range(2):
        assert env.removed[l] == rem0[l] | pruned[l]
    assert alive_edges(g, env.covered, env.removed) == final
