"""The degree-cost MultiDismantler agent, inference path (drop-in for
``D/MultiDismantler_torch.py``; D/ = ``code/MultiDismantler_degree_cost``).

Same device path as :mod:`mdcommunity_amd.agent` (Q network, arg-max, cover and mutual-LMCC
cascade in ``libmdroll.so``) with the variant's differences:

* node inputs ``[w_l(v), 1.0]`` from the original degrees (``D/PrepareBatchGraph.py:133-136``,
  ``D/graph.py:91-115``) instead of the residual-degree features — passed to the device as
  ``node_w`` (first layer computed once per graph on the host in the reference's fp32 order);
* weighted reward ``-rank/max_rank * (w0[a]/W0 + w1[a]/W1)/2`` and ``MaxCCList`` entries
  ``rank/max_rank`` (``D/mvc_env.py:75-134``);
* ``GetSol`` returns the summed node cost (``:734-768``), ``Evaluate`` skips graphs whose
  initial LMCC is 1 (``:540-577``), ``EvaluateRealData`` writes ``Solution_`` /
  ``NormalizedLMCC_`` / ``Cost_`` files (``:623-681``).
"""
import os
import sys
import time

import numpy as np

from . import _lib, agent as _agent, engine as _engine, graph as _graph


class MultiDismantler(_agent.MultiDismantler):
    cost_mode = _lib.MD_COST_DEGREE

    def LoadModel(self, model_path):  # noqa: N802
        super().LoadModel(model_path if model_path is not None else _engine.DEFAULT_DEGREE)

    def _node_w(self, g):
        return _graph.node_weight_array([g])

    def _batch_node_w(self, graphs):
        return _graph.node_weight_array(graphs)

    def _replay_scores(self, g, seq, ranks):
        """score / MaxCCList with the variant's float64 expressions (D/mvc_env.py:75-88,127-134)."""
        env = self.test_env
        env.action_list = list(seq)
        env.score = 0.0
        env.MaxCCList = [1]
        for a, rank in zip(seq, ranks):
            r_t = env._reward(a, rank)
            env.score += -1 * r_t
            env.MaxCCList.append(rank / (g.max_rank))
        env._refresh()

    def _device_rollout(self, g, step):
        _graph.ensure_degree_weights(g)
        return super()._device_rollout(g, step)

    def GetSol(self, gid, step=1):  # noqa: N802
        """(score, solution, summed node cost) (D/MultiDismantler_torch.py:734-768)."""
        g = self.TestSet.Get(gid)
        seq, ranks = self._device_rollout(g, step)
        self._replay_scores(g, seq, ranks)
        total_weight0 = sum(g.weights[0].values())
        total_weight1 = sum(g.weights[1].values())
        total_cost_value = 0
        for cost_node in seq:
            total_cost_value += (g.weights[0][cost_node] / total_weight0 + g.weights[1][cost_node] / total_weight1) / 2.0
        return self.test_env.score, seq, total_cost_value

    def GetSolution(self, gid, step=1):  # noqa: N802
        """(solution, score, MaxCCList) (D/MultiDismantler_torch.py:683-706)."""
        g = self.TestSet.Get(gid)
        seq, ranks = self._device_rollout(g, step)
        self._replay_scores(g, seq, ranks)
        _agent.print_iterations(len(seq), step)
        return seq, self.test_env.score, self.test_env.MaxCCList

    def GetSolBatch(self, graphs, step=1):
        """Batched rollouts (configs 3 / 5) with the variant's weighted score."""
        for g in graphs:
            _graph.ensure_degree_weights(g)
        eng = self.engine
        eng.load_graphs([(g.num_nodes, g.edges[0], g.edges[1]) for g in graphs],
                        node_w=self._batch_node_w(graphs))
        mr = eng.reset()
        outs = eng.rollout(step=step)
        res = []
        for g, m, (seq, ranks) in zip(graphs, mr, outs):
            tw0 = sum(g.weights[0].values())
            tw1 = sum(g.weights[1].values())
            score = 0.0
            for a, r in zip(seq, ranks):
                score += -1 * (-int(r) / (g.max_rank) * (g.weights[0][int(a)] / tw0 + g.weights[1][int(a)] / tw1) / 2.0)
            res.append((score, [int(a) for a in seq], [int(r) for r in ranks]))
        self.test_env.graph = None
        return res

    def Evaluate(self, data_test, data_test_name, dirt, model_file=None, data_root="../../data"):  # noqa: N802
        """testSynthetic harness (D/MultiDismantler_torch.py:540-577)."""
        print("The best model is :%s" % (model_file if model_file is not None
                                          else _engine.resolve_model(None, self.cost_mode)))
        sys.stdout.flush()
        self.LoadModel(model_file)
        n_test = 2 if os.getenv("SMOKE_TEST", "0").strip().lower() in ("1", "true", "yes") else 20
        scores, times, costs = [], [], []
        j = 0
        for i in range(n_test):
            base = os.path.join(data_root, "synthetic", dirt, "syn_%s" % data_test_name)
            a1 = np.load(os.path.join(base, "adj1_%s.npy" % i))
            a2 = np.load(os.path.join(base, "adj2_%s.npy" % i))
            g = _graph.Graph_test.from_edges(a1.shape[0], np.argwhere(np.triu(a1) > 0), np.argwhere(np.triu(a2) > 0))
            if g.max_rank == 1:
                continue
            self.InsertGraph(g, is_test=True)
            t1 = time.time()
            val, sol, cost_value = self.GetSol(j)
            t2 = time.time()
            costs.append(cost_value)
            scores.append(val)
            times.append(t2 - t1)
            j += 1
        self.ClearTestGraphs()
        return np.mean(scores), np.std(scores), np.mean(times), np.std(times), np.mean(costs)

    def EvaluateRealData(self, model_file, data_test, save_dir, stepRatio, num_nodes, layers,  # noqa: N802,N803
                         data_root="../../data"):
        """testReal harness (D/MultiDismantler_torch.py:623-681): Solution_, NormalizedLMCC_,
        Cost_ files."""
        test_name = data_test.split("/")[-1]
        save_dir_local = save_dir + "/StepRatio_%.4f" % stepRatio
        if not os.path.exists(save_dir_local):
            os.mkdir(save_dir_local)
        stem = test_name.split(".")[0]
        f1 = "%s/%s_%s_%s%s.%s" % (save_dir_local, "Solution", stem, layers[0], layers[1], "txt")
        f2 = "%s/%s_%s_%s%s.%s" % (save_dir_local, "NormalizedLMCC", stem, layers[0], layers[1], "txt")
        f3 = "%s/%s_%s_%s%s.%s" % (save_dir_local, "Cost", stem, layers[0], layers[1], "txt")
        _, gl = self.read_multiplex(os.path.join(data_root, "real", test_name), num_nodes)
        g = _graph.Graph_test.from_edges(num_nodes, gl[layers[0] - 1], gl[layers[1] - 1])
        _graph.ensure_degree_weights(g)
        with open(f1, "w") as fo:
            print("testing")
            sys.stdout.flush()
            step = max(int(stepRatio * g.num_nodes), 1) if stepRatio > 0 else 1
            self.InsertGraph(g, is_test=True)
            t1 = time.time()
            solution, score, maxcc = self.GetSolution(0, step)
            t2 = time.time()
            solution_time = t2 - t1
            for a in solution:
                fo.write("%d\n" % a)
        with open(f2, "w") as fo:
            for j in range(g.num_nodes):
                if j < len(solution):
                    fo.write("%.8f\n" % maxcc[j])
                else:
                    fo.write("%.8f\n" % (1 / g.max_rank))
        nodes = list(range(g.num_nodes))
        remain_nodes = list(set(nodes) ^ set(solution))
        total_weight0 = sum(g.weights[0].values())
        total_weight1 = sum(g.weights[1].values())
        cost = [0]
        total_cost = 0
        for node in solution + remain_nodes[:-1]:
            total_cost += (g.weights[0][node] / total_weight0 + g.weights[1][node] / total_weight1) / 2.0
            cost.append(total_cost)
        cost.append(score)
        with open(f3, "w") as fo:
            for c in cost:
                fo.write("%.8f\n" % c)
        self.ClearTestGraphs()
        return solution, solution_time, score
