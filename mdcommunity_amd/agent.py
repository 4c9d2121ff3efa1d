"""The MultiDismantler agent, inference path (drop-in for ``U/MultiDismantler_torch.py``).

Kept surface (``U/MultiDismantler_torch.py``): ``LoadModel`` (:791-797), ``InsertGraph`` /
``ClearTestGraphs`` (:162-178), ``PredictWithCurrentQNet`` (:304-306 -> ``Predict``
:263-302), ``GetSol`` (:759-784), ``GetSolution`` (:711-736), ``Evaluate`` (:563-600),
``read_multiplex`` (:602-635), ``EvaluateRealData`` (:645-709), ``argMax`` (:799-807).
Everything per step (Q network, arg-max, cover + mutual-LMCC cascade) runs on the MI355X in
``libmdroll.so``; the host only keeps the reference's bookkeeping (score, MaxCCList, output
files) with the reference's own float64 expressions.  Training (``Fit``, ``Train``,
replay memory) is out of scope.

``GetSolBatch`` is the batched extension: many graphs in one device launch sequence
(BASELINE configs 3 and 5).
"""
import os
import sys
import time

import numpy as np

from . import _lib, engine as _engine, graph as _graph
from .mvc_env import MvcEnv

INF = 2147483647 / 2          # U/MultiDismantler_torch.py:60
NUM_MAX = 50                  # :52
BATCH_SIZE = 64               # :54


class MultiDismantler:
    cost_mode = _lib.MD_COST_UNIT

    def __init__(self, device=0):
        self.device = device
        self.TestSet = _graph.GSet()
        self.TrainSet = _graph.GSet()
        self.ngraph_test = 0
        self.ngraph_train = 0
        self._weights = None
        self._engine = None
        self.test_env = MvcEnv(NUM_MAX, cost_mode=self.cost_mode)
        self.model_file = None
        # the reference constructor's log lines (U/MultiDismantler_torch.py:107,124)
        print("CUDA:", _lib.device_count() > 0)
        print("Total number of MultiDismantler_net parameters: {}".format(_lib.MD_WEIGHT_FLOATS))

    # ---------------------------------------------------------------- model / graphs
    @property
    def engine(self):
        if self._engine is None:
            if self._weights is None:
                self.LoadModel(None)
            self._engine = _lib.Engine(self._weights, device=self.device, cost_mode=self.cost_mode)
            self.test_env.attach(self._engine)
        return self._engine

    def LoadModel(self, model_path):  # noqa: N802
        """Load a checkpoint (reference .ckpt via torch.load(weights_only=True), or .npz)."""
        self.model_file = _engine.resolve_model(model_path, self.cost_mode)
        self._weights = _engine.load_weights(self.model_file)
        if self._engine is not None:
            self._engine.set_weights(self._weights)
        print("restore model from file successfully")

    def InsertGraph(self, g, is_test):  # noqa: N802
        if is_test:
            self.TestSet.InsertGraph(self.ngraph_test, g)
            self.ngraph_test += 1
        else:
            self.TrainSet.InsertGraph(self.ngraph_train, g)
            self.ngraph_train += 1

    def ClearTestGraphs(self):  # noqa: N802
        self.ngraph_test = 0
        self.TestSet.Clear()

    def ClearTrainGraphs(self):  # noqa: N802
        self.ngraph_train = 0
        self.TrainSet.Clear()

    # ---------------------------------------------------------------- prediction
    def _masked_row(self, q32):
        q = q32.astype(np.float64)
        q[~np.isfinite(q32)] = -INF
        return q

    def PredictWithCurrentQNet(self, g_list, covered, remove_edges):  # noqa: N802
        """Masked float64 Q rows, one per graph (Predict, :263-302).  States other than the
        live environment's are loaded with md_set_state first (no MCC, as in the reference)."""
        eng = self.engine
        env = self.test_env
        out = []
        for g, cov, rem in zip(g_list, covered, remove_edges):
            live_state = env.graph is g and cov is env.action_list
            if not live_state:
                env.graph = None
                eng.load_graphs([(g.num_nodes, g.edges[0], g.edges[1])], node_w=self._node_w(g))
                c = np.zeros(g.num_nodes, np.uint8)
                c[list(cov)] = 1
                rs = []
                for l in range(2):
                    rs.append(np.asarray([(int(u), int(v)) in rem[l] for u, v in g.edges[l]], dtype=np.uint8))
                eng.set_state(0, c, rs[0], rs[1])
            q, _, _, _ = eng.predict()
            out.append(self._masked_row(q[: g.num_nodes]))
        return out

    def PredictWithSnapshot(self, g_list, covered, remove_edges):  # noqa: N802
        return self.PredictWithCurrentQNet(g_list, covered, remove_edges)

    def _node_w(self, g):
        return None

    # ---------------------------------------------------------------- rollouts
    def _device_rollout(self, g, step):
        env = self.test_env
        env.attach(self.engine)
        env.s0(g)
        out = self.engine.rollout(step=step)
        seq, ranks = out[0]
        return [int(a) for a in seq], [int(r) for r in ranks]

    def _replay_scores(self, g, seq, ranks):
        """score / MaxCCList in the reference's order of float64 operations (U/mvc_env.py:86-87)."""
        env = self.test_env
        env.action_list = list(seq)
        env.score = 0.0
        env.MaxCCList = [1]
        for a, rank in zip(seq, ranks):
            r_t = env._reward(a, rank)
            env.score += -1 * r_t
            env.MaxCCList.append(-1 * r_t * g.num_nodes)
        env._refresh()

    def GetSol(self, gid, step=1):  # noqa: N802
        """Rollout of test graph gid (:759-784) -> (score, solution, len(sol)/N)."""
        g = self.TestSet.Get(gid)
        seq, ranks = self._device_rollout(g, step)
        self._replay_scores(g, seq, ranks)
        return self.test_env.score, seq, len(seq) / g.num_nodes

    def GetSolution(self, gid, test_name=None, step=1):  # noqa: N802
        """testReal rollout (:711-736) -> (solution, score, MaxCCList)."""
        g = self.TestSet.Get(gid)
        seq, ranks = self._device_rollout(g, step)
        self._replay_scores(g, seq, ranks)
        print_iterations(len(seq), step)
        return seq, self.test_env.score, self.test_env.MaxCCList

    def GetSolBatch(self, graphs, step=1):
        """Batched rollouts of many graphs in one engine (configs 3 / 5).  Returns a list of
        (score, solution, ranks) in the reference's score arithmetic."""
        eng = self.engine
        eng.load_graphs([(g.num_nodes, g.edges[0], g.edges[1]) for g in graphs],
                        node_w=self._batch_node_w(graphs))
        mr = eng.reset()
        outs = eng.rollout(step=step)
        res = []
        for g, m, (seq, ranks) in zip(graphs, mr, outs):
            if getattr(g, "_max_rank", None) is None:
                g.max_rank = int(m)
            score = 0.0
            for r in ranks:
                score += -1 * (-float(r) / (g.max_rank * float(g.num_nodes)))
            res.append((score, [int(a) for a in seq], [int(r) for r in ranks]))
        self.test_env.graph = None
        return res

    def _batch_node_w(self, graphs):
        return None

    def argMax(self, scores):  # noqa: N802
        n = len(scores)
        pos, best = -1, -10000000
        for i in range(n):
            if pos == -1 or scores[i] > best:
                pos, best = i, scores[i]
        return pos

    # ---------------------------------------------------------------- harnesses
    def Evaluate(self, data_test, data_test_name, data_type, model_file=None, data_root="../../data"):  # noqa: N802
        """testSynthetic harness (:563-600): 20 graphs adj{1,2}_<i>.npy per size."""
        print("The best model is :%s" % (model_file if model_file is not None
                                          else _engine.resolve_model(None, self.cost_mode)))
        sys.stdout.flush()
        self.LoadModel(model_file)
        n_test = 2 if os.getenv("SMOKE_TEST", "0").strip().lower() in ("1", "true", "yes") else 20
        scores, times, costs = [], [], []
        for i in range(n_test):
            base = os.path.join(data_root, "synthetic", data_type, "syn_%s" % data_test_name)
            a1 = np.load(os.path.join(base, "adj1_%s.npy" % i))
            a2 = np.load(os.path.join(base, "adj2_%s.npy" % i))
            g = _graph.Graph_test.from_edges(a1.shape[0], np.argwhere(np.triu(a1) > 0), np.argwhere(np.triu(a2) > 0))
            self.InsertGraph(g, is_test=True)
            t1 = time.time()
            val, sol, cost = self.GetSol(i)
            t2 = time.time()
            scores.append(val)
            times.append(t2 - t1)
            costs.append(cost)
        self.ClearTestGraphs()
        return np.mean(scores), np.std(scores), np.mean(times), np.std(times), np.mean(costs)

    def read_multiplex(self, path, N):
        """Parse ``layer u v [w]`` lines (1-based ids, self-loops dropped; :602-635) into
        per-layer edge lists in networkx insertion order."""
        layers = []
        cur, adj, order = None, None, None

        def flush():
            if adj is not None:
                layers.append(_edges_in_nx_order(N, order))

        with open(path, "r") as lines:
            cur_id = 1
            adj, order = set(), []
            for ln in lines:
                el = ln.strip(" \n").split(" ")
                lid = int(el[0])
                if cur_id != lid:
                    flush()
                    adj, order = set(), []
                    cur_id = lid
                u, v = int(el[1]) - 1, int(el[2]) - 1
                if u == v:
                    continue
                key = (min(u, v), max(u, v))
                if key not in adj:
                    adj.add(key)
                    order.append((u, v))
            flush()
        return None, layers

    def EvaluateRealData(self, model_file, data_test, save_dir, stepRatio, num_nodes, layers, data_root="../../data"):  # noqa: N802,N803
        """testReal harness (:645-709): writes Soluion_*, NormalizedLMCC_* (unit cost)."""
        test_name = data_test.split("/")[-1]
        save_dir_local = save_dir + "/StepRatio_%.4f" % stepRatio
        if not os.path.exists(save_dir_local):
            os.mkdir(save_dir_local)
        stem = test_name.split(".")[0]
        f1 = "%s/%s_%s_%s%s.%s" % (save_dir_local, "Soluion", stem, layers[0], layers[1], "txt")
        f2 = "%s/%s_%s_%s%s.%s" % (save_dir_local, "NormalizedLMCC", stem, layers[0], layers[1], "txt")
        _, gl = self.read_multiplex(os.path.join(data_root, "real", test_name), num_nodes)
        g = _graph.Graph_test.from_edges(num_nodes, gl[layers[0] - 1], gl[layers[1] - 1])
        mcc_avg = [0] * g.num_nodes
        scores = []
        with open(f1, "w") as fo:
            print("testing")
            sys.stdout.flush()
            step = max(int(stepRatio * g.num_nodes), 1) if stepRatio > 0 else 1
            self.InsertGraph(g, is_test=True)
            t1 = time.time()
            sol, score, maxcc = self.GetSolution(0, test_name, step)
            mcc_avg = [mcc_avg[i] + maxcc[i] for i in range(min(len(mcc_avg), len(maxcc)))]
            scores.append(score)
            t2 = time.time()
            solution_time = t2 - t1
            score_mean = np.mean(scores)
            print(score_mean)
            score_std = np.std(scores)
            for a in sol:
                fo.write("%d\n" % a)
        with open(f2, "w") as fo:
            for j in range(g.num_nodes):
                if j < len(mcc_avg):
                    fo.write("%.8f\n" % (float(mcc_avg[j] / 1)))
                else:
                    fo.write("%.8f\n" % (1 / g.max_rank))
        with open(f2, "a") as fo:
            fo.write("%.8f\n" % score_mean)
            fo.write("%.8f\n" % score_std)
        self.ClearTestGraphs()
        return sol, solution_time, score


def print_iterations(removals, step):
    """GetSolution's log (U/MultiDismantler_torch.py:721, D/MultiDismantler_torch.py:692): one
    ``Iteration:%d`` line per prediction of the loop.  Every prediction but the last applies
    `step` actions (an iteration stops short only when the graph became terminal), so a rollout
    of `removals` removals made ceil(removals / step) predictions."""
    for it in range(-(-removals // step)):
        print("Iteration:%d" % it)


def _edges_in_nx_order(n, order):
    """Edge list of a networkx Graph built by add_node(0..n-1) then add_edge in `order`:
    G.edges() visits nodes in id order, each node's neighbours in insertion order, and
    yields every edge once from its first-visited endpoint."""
    nbrs = [[] for _ in range(n)]
    for u, v in order:
        nbrs[u].append(v)
        nbrs[v].append(u)
    seen = np.zeros(n, bool)
    out = []
    for u in range(n):
        for v in nbrs[u]:
            if not seen[v]:
                out.append((u, v))
        seen[u] = True
    return np.asarray(out, dtype=np.int32).reshape(-1, 2)
