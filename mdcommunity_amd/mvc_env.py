"""Rollout environment (drop-in for ``U/mvc_env.py`` / ``D/mvc_env.py``).

``MvcEnv`` keeps the reference's attributes and methods (``s0``, ``stepWithoutReward``,
``isTerminal``, ``getReward``, ``score``, ``MaxCCList``, ``action_list``, ``covered_set``,
``remove_edge``, ``numCoveredEdges``) while the state lives on the device: covering a node
and the mutual-LMCC cascade run in ``libmdroll.so`` (``md_step``).  ``covered_set`` and
``remove_edge`` are materialised from the device state on access.
"""
import numpy as np

from . import _lib


class MvcEnv:
    def __init__(self, norm, engine=None, cost_mode=_lib.MD_COST_UNIT):
        self.norm = norm
        self.graph = None
        self._engine = engine
        self._own_engine = engine is None
        self.cost_mode = cost_mode
        self.action_list = []
        self.MaxCCList = [1]
        self.score = 0.0
        self.flag = 0
        self._counters = np.zeros(6, np.int32)
        self._wsum = None

    # -- device plumbing
    @property
    def engine(self):
        if self._engine is None:
            self._engine = _lib.Engine(np.zeros(_lib.MD_WEIGHT_FLOATS, np.float32), cost_mode=self.cost_mode)
        return self._engine

    def attach(self, engine):
        self._engine = engine
        self._own_engine = False

    def _load(self, g):
        nw = None
        if self.cost_mode == _lib.MD_COST_DEGREE:
            from .graph import node_weight_array
            nw = node_weight_array([g])
        self.engine.load_graphs([(g.num_nodes, g.edges[0], g.edges[1])], node_w=nw)

    # -- reference API
    def s0(self, g):
        """Reset on graph g and run the initial mutual-LMCC prune (U/mvc_env.py:31-52)."""
        self.graph = g
        self._load(g)
        mr = self.engine.reset()
        if getattr(g, "_max_rank", None) is None:
            g.max_rank = int(mr[0])
        self.action_list = []
        self.MaxCCList = [1]
        self.score = 0.0
        self.flag = 1
        self._refresh()

    def _refresh(self):
        self._counters = self.engine.get_state(0)[3]

    def stepWithoutReward(self, a):  # noqa: N802
        """Cover node a, cascade, accumulate the reward (U/mvc_env.py:74-87)."""
        assert self.graph is not None
        a = int(a)
        assert a not in self.action_list
        lm, _ = self.engine.step(np.array([a], np.int32))
        self.action_list.append(a)
        self._refresh()
        r_t = self._reward(a, int(lm[0]))
        self.score += -1 * r_t
        if self.cost_mode == _lib.MD_COST_UNIT:
            self.MaxCCList.append(-1 * r_t * self.graph.num_nodes)
        else:
            self.MaxCCList.append(float(lm[0]) / self.graph.max_rank)
        return r_t

    def _reward(self, a, rank):
        g = self.graph
        if self.cost_mode == _lib.MD_COST_UNIT:
            return -float(rank) / (g.max_rank * float(g.num_nodes))  # U/mvc_env.py:133-137
        w0, w1 = g.weights[0], g.weights[1]
        if self._wsum is None or self._wsum[0] is not g:
            self._wsum = (g, sum(w0.values()), sum(w1.values()))
        return -rank / (g.max_rank) * (w0[a] / self._wsum[1] + w1[a] / self._wsum[2]) / 2.0  # D/mvc_env.py:127-134

    def getReward(self, a):  # noqa: N802
        return self._reward(a, int(self._counters[4]))

    def isTerminal(self):  # noqa: N802
        """U/mvc_env.py:128-131: some layer has no alive edge left."""
        assert self.graph is not None
        return bool(self._counters[5])

    @property
    def numCoveredEdges(self):  # noqa: N802
        return [int(self._counters[0]), int(self._counters[1])]

    @property
    def covered_set(self):
        return set(self.action_list)

    @property
    def remove_edge(self):
        """Edges pruned by the MCC cascade, both orientations (U/Mcc.py:8-10)."""
        _, r0, r1, _ = self.engine.get_state(0)
        out = []
        for l, r in enumerate((r0, r1)):
            s = set()
            for u, v in self.graph.edges[l][r]:
                s.add((int(u), int(v)))
                s.add((int(v), int(u)))
            out.append(s)
        return out

    def getMaxConnectedNodesNum(self, a=None):  # noqa: N802
        return float(self._counters[4])
