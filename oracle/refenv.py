"""Reference-shaped environment, featuriser and rollout — TEST INFRASTRUCTURE ONLY.

Restates, per removal step, what the reference does on the host:

* mutual-LMCC cascade ``U/Mcc.py:3-38`` (networkx components, alternate edge deletion
  until both layers' partitions agree) and the env bookkeeping of ``MvcEnv``
  (``U/mvc_env.py:31-52`` s0, ``:74-87`` stepWithoutReward, ``:128-137`` isTerminal/getReward,
  ``:140-162`` getMaxConnectedNodesNum);
* featurisation ``U/PrepareBatchGraph.py:35-74`` (get_status_info) and ``:76-177``
  (Setup_graph_input: ascending live-node compaction, in_edges aggregation order, aux
  features), rebuilt from scratch in Python every step as the reference does;
* the selection ``np.argsort(-q)[:step]`` of ``U/MultiDismantler_torch.py:725,769`` on the
  masked float64 Q row built like ``Predict`` (``:286-300``, mask ``-(2147483647/2)``, ``:60``).

It is deliberately reference-shaped (Python edge scans + torch-CPU forward + networkx
BFS every step) so that ``bench.py`` can time it as the CPU baseline on the GPU box,
where the reference itself cannot travel.
"""
import networkx as nx
import numpy as np

from . import refmodel

MASK = -(2147483647 / 2)


class RefGraph:
    """Graph_test (U/graph.py:69-84; D/graph.py:72-115 adds the degree weights) from two
    ordered edge lists on nodes 0..n-1."""

    def __init__(self, n, edges0, edges1):
        self.num_nodes = int(n)
        self.edge_list = [[(int(u), int(v)) for u, v in np.asarray(e).reshape(-1, 2)] for e in (edges0, edges1)]
        self.num_edges = [len(self.edge_list[0]), len(self.edge_list[1])]
        self.adj = [[[] for _ in range(self.num_nodes)] for _ in range(2)]
        for l in range(2):
            for u, v in self.edge_list[l]:
                self.adj[l][u].append(v)
                self.adj[l][v].append(u)
        g1, g2 = self.nx_layers()
        self.max_rank = lmcc_size(mutual_components(g1, g2, [set(), set()]))
        # D/graph.py:91-115 cal_degree: original degree / max degree, per layer (only when
        # max_rank != 1 there; the weights are unused otherwise)
        self.weights = [[], []]
        if self.max_rank != 1:
            for l in range(2):
                d = [len(self.adj[l][v]) for v in range(self.num_nodes)]
                m = max(d)
                self.weights[l] = [x / m for x in d]

    def nx_layers(self, covered=(), removed=(set(), set())):
        out = []
        for l in range(2):
            g = nx.Graph()
            g.add_nodes_from(range(self.num_nodes))
            for u, v in self.edge_list[l]:
                if u not in covered and v not in covered and (u, v) not in removed[l]:
                    g.add_edge(u, v)
            out.append(g)
        return out


def _components(g):
    comps = [set(c) for c in nx.connected_components(g)]
    label = {}
    for i, c in enumerate(comps):
        for v in c:
            label[v] = i
    return comps, label


def _prune(g, label, removed):
    for u, v in list(g.edges):
        if label.get(u, -1) != label.get(v, -2):
            g.remove_edge(u, v)
            removed.add((u, v))
            removed.add((v, u))


def mutual_components(g1, g2, removed):
    """U/Mcc.py:30-38: prune layer 2 by layer-1 components, then layer 1 by layer-2
    components, until the two partitions (as ordered component lists) agree."""
    c1, lab1 = _components(g1)
    c2, lab2 = _components(g2)
    while c1 != c2:
        _prune(g2, lab1, removed[1])
        c2, lab2 = _components(g2)
        _prune(g1, lab2, removed[0])
        c1, lab1 = _components(g1)
    return c1


def lmcc_size(comps):
    return len(max(comps, key=len, default=()))


class RefEnv:
    """MvcEnv: unit cost (U/mvc_env.py) or degree cost (D/mvc_env.py:75-134)."""

    def __init__(self, graph, cost="unit"):
        self.graph = graph
        self.cost = cost
        self.covered = set()
        self.action_list = []
        self.removed = [set(), set()]
        self.num_covered = [0, 0]
        self.score = 0.0
        self.maxcc = [1]
        self.ranks = []
        self.g1, self.g2 = graph.nx_layers()
        mutual_components(self.g1, self.g2, self.removed)

    def terminal(self):
        g = self.graph
        return any(g.num_edges[l] == self.num_covered[l] + len(self.removed[l]) / 2 for l in range(2))

    def step(self, a):
        assert a not in self.covered
        self.covered.add(a)
        self.action_list.append(a)
        for l in range(2):
            for nb in self.graph.adj[l][a]:
                if nb not in self.covered and (nb, a) not in self.removed[l]:
                    self.num_covered[l] += 1
        self.g1.remove_node(a)
        self.g2.remove_node(a)
        g = self.graph
        if self.cost == "degree":
            rank = lmcc_size(mutual_components(self.g1, self.g2, self.removed))
            tw0 = sum(g.weights[0])
            tw1 = sum(g.weights[1])
            r_t = -rank / (g.max_rank) * (g.weights[0][a] / tw0 + g.weights[1][a] / tw1) / 2.0
            self.score += -1 * r_t
            self.maxcc.append(rank / (g.max_rank))
        else:
            rank = float(lmcc_size(mutual_components(self.g1, self.g2, self.removed)))
            r_t = -rank / (g.max_rank * float(g.num_nodes))
            self.score += -1 * r_t
            self.maxcc.append(-1 * r_t * g.num_nodes)
        self.ranks.append(int(rank))
        return int(rank)


def featurize(graph, covered, removed):
    """get_status_info + Setup_graph_input for one graph: live-node ids (ascending),
    per-layer residual degree of each live node, n2n COO in in_edges order, aux feats."""
    n = graph.num_nodes
    live = [[False] * n, [False] * n]
    counter = [0, 0]
    twohop = [0, 0]
    for l in range(2):
        seen = {}
        for u, v in graph.edge_list[l]:
            if (u, v) in removed[l]:
                continue
            if u in covered or v in covered:
                counter[l] += 1
                continue
            live[l][u] = live[l][v] = True
            for x in (u, v):
                k = seen.get(x, 0)
                twohop[l] += k
                seen[x] = k + 1
    assert live[0] == live[1], "live node sets differ between layers (U/PrepareBatchGraph.py:73)"
    ids = [v for v in range(n) if live[0][v]]
    pos = {v: i for i, v in enumerate(ids)}
    coo = []
    deg = []
    for l in range(2):
        inn = [[] for _ in ids]
        for u, v in graph.edge_list[l]:
            if (u, v) in removed[l] or u not in pos or v not in pos:
                continue
            inn[pos[v]].append(pos[u])
            inn[pos[u]].append(pos[v])
        rows = [i for i, lst in enumerate(inn) for _ in lst]
        cols = [x for lst in inn for x in lst]
        coo.append((np.asarray(rows, dtype=np.int64), np.asarray(cols, dtype=np.int64)))
        deg.append([len(set(lst)) for lst in inn])
    nn = float(len(covered)) / n
    aux = [[nn, counter[l] / graph.num_edges[l], twohop[l] / (n * n), 1.0] for l in range(2)]
    return ids, deg, coo, aux, counter


def predict(weights, graph, covered, removed, cost="unit"):
    """Masked float64 Q row over all node ids (Predict, U/MultiDismantler_torch.py:263-302).
    Degree cost: node inputs [weight, 1.0] of the live nodes (D/PrepareBatchGraph.py:133-136)."""
    ids, deg, coo, aux, _ = featurize(graph, covered, removed)
    row = np.full(graph.num_nodes, MASK, dtype=np.float64)
    if ids:
        feat = None
        if cost == "degree":
            feat = [[[graph.weights[l][v], 1.0] for v in ids] for l in range(2)]
        q = refmodel.forward(weights, deg, coo, aux, node_feat=feat)
        row[np.asarray(ids)] = q.astype(np.float64)
    for k in covered:
        row[k] = MASK
    return row


def rollout(weights, graph, step=1, on_predict=None, cost="unit"):
    """GetSol (U/MultiDismantler_torch.py:759-784; D :734-768): returns (score, sequence,
    ranks, maxcc)."""
    env = RefEnv(graph, cost)
    sol = []
    t = 0
    while not env.terminal():
        q = predict(weights, graph, env.covered, env.removed, cost)
        if on_predict is not None:
            on_predict(t, q, env)
        t += 1
        for a in np.argsort(-q)[:step]:
            if env.terminal():
                break
            env.step(int(a))
            sol.append(int(a))
    return env.score, sol, env.ranks, env.maxcc
