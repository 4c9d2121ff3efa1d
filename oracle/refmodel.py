"""Q network forward of the reference, op for op in torch-CPU — TEST INFRASTRUCTURE ONLY.

Restates ``MultiDismantler_net.test_forward`` (``U/MultiDismantler_net_graphsage.py:243-394``)
and ``BitwiseMultipyLogis.forward`` / ``LogisticVector`` (``U/MRGNN/mutil_layer_weight.py:252-313``)
for ONE graph, keeping every torch op, operand order and tensor shape of the reference so
that on the build host (same torch / MKL) the result is bit-identical to the reference's.
The sparse products go through :func:`spmm`, the published algorithm of
``torch_sparse.spmm`` 0.6.x (``index_select`` of the columns, scale by the values, then a
sequential ``scatter_add`` over the rows).
"""
import numpy as np
import torch
import torch.nn.functional as F

EMB = 64


def spmm(row, col, value, m, mat):
    """torch_sparse.spmm(index, value, m, n, matrix) (R/uv.lock:1498, call sites
    U/MultiDismantler_net_graphsage.py:290-298,350-351,377-378)."""
    src = mat.index_select(0, col) * value.unsqueeze(-1)
    out = torch.zeros((m, src.size(1)), dtype=src.dtype)
    return out.scatter_add_(0, row.unsqueeze(-1).expand_as(src), src)


class RefWeights:
    """The 14 tensors of the reference state_dict as fp32 torch tensors."""

    def __init__(self, arrays):
        # The reference runs inference with autograd ON and requires_grad parameters
        # (U/MultiDismantler_torch.py:112-121, no torch.no_grad()); that selects different
        # (fused vs. unfused) CPU kernels for F.linear on 3-D inputs, so the oracle does too.
        t = {k: torch.nn.Parameter(torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)))
             for k, v in arrays.items()}
        self.w_n2l = t["w_n2l"]
        self.p1 = t["p_node_conv"]
        self.p2 = t["p_node_conv2"]
        self.p3 = t["p_node_conv3"]
        self.h1 = t["h1_weight"]
        self.last_w = t["last_w"] if "last_w" in t else t["h2_weight"]
        self.cross = t["cross_product"]
        self.wl1 = t["w_layer1"]
        self.wl2 = t["w_layer2"]
        self.trans = t["layerNodeAttention_weight.trans"]
        self.tbias = t["layerNodeAttention_weight.bias"]
        self.lw = t["layerNodeAttention_weight.logis.parameter.weight"]
        self.lb = t["layerNodeAttention_weight.logis.parameter.bias"]

    @classmethod
    def load(cls, path):
        with np.load(path, allow_pickle=False) as z:
            return cls({k: z[k] for k in z.files})


def _attention(w, embeds, layer):
    """BitwiseMultipyLogis.forward(node_features, nodes, layer_predict), metapath_number=2."""
    rows = embeds[0].size(0)
    feats = torch.zeros((2, rows, EMB))
    for k in range(2):
        feats[k] = torch.tanh(torch.matmul(embeds[k], w.trans) + w.tbias)
    per_node = torch.transpose(feats, 0, 1)                      # [rows, 2, 64]
    other = [k for k in range(2) if k != layer]
    sem = torch.zeros_like(per_node)
    sem[:, other] = per_node[:, other] * per_node[:, layer].unsqueeze(1)
    sem[:, layer] = per_node[:, layer] * per_node[:, layer]
    gate = torch.sigmoid(F.linear(sem, w.lw, w.lb)).squeeze()    # LogisticVector
    gate = gate.reshape(rows, 2)
    gate = F.softmax(gate, dim=1)
    z = torch.zeros(rows, EMB)
    for k in other:
        z = z + gate[:, k].unsqueeze(1) * per_node[:, k]
    return feats[layer] + z


def forward(w, deg, n2n, aux, max_bp_iter=3, node_feat=None):
    """Q values of the live nodes of one graph.

    deg      [2][n] residual degree of each live node per layer (compact ascending order)
    n2n      [2] (row, col) int64 COO of the residual adjacency in in_edges order
    aux      [2][4] float32 aux features (U/PrepareBatchGraph.py:92-101)
    node_feat optional [2][n][2] node inputs (degree-cost variant); default = unit cost
    returns  q [n] float32
    """
    n = len(deg[0])
    node_input = torch.zeros((2, n, 2), dtype=torch.float)
    if node_feat is None:
        for l in range(2):
            d = torch.as_tensor(np.asarray(deg[l], dtype=np.float32)).reshape(n, 1)
            dmax, _ = torch.max(d, dim=0)
            dn = d / dmax
            node_input[l] = torch.cat((dn, dn), axis=1)
    else:
        node_input = torch.as_tensor(np.asarray(node_feat, dtype=np.float32))
    y_input = torch.ones((2, 1, 2), dtype=torch.float)
    sub_row = torch.zeros(n, dtype=torch.long)
    sub_col = torch.arange(n, dtype=torch.long)
    ones_n = torch.ones(n)
    embeds = []
    for l in range(2):
        row = torch.as_tensor(n2n[l][0], dtype=torch.long)
        col = torch.as_tensor(n2n[l][1], dtype=torch.long)
        val = torch.ones(row.numel())
        h = F.normalize(torch.relu(torch.matmul(node_input[l], w.w_n2l)), p=2, dim=1)
        y = F.normalize(torch.relu(torch.matmul(y_input[l], w.w_n2l)), p=2, dim=1)
        for _ in range(max_bp_iter):
            pool = spmm(row, col, val, n, h)
            node_lin = torch.matmul(pool, w.p1)
            ypool = spmm(sub_row, sub_col, ones_n, 1, h)
            y_node_lin = torch.matmul(ypool, w.p1)
            cur_lin = torch.matmul(h, w.p2)
            h = F.normalize(torch.relu(torch.matmul(torch.concat([node_lin, cur_lin], 1), w.p3)), p=2, dim=1)
            y_cur_lin = torch.matmul(y, w.p2)
            y = F.normalize(torch.relu(torch.matmul(torch.concat([y_node_lin, y_cur_lin], 1), w.p3)), p=2, dim=1)
        embeds.append(torch.cat((h, y), axis=0))
    msg = torch.zeros(2, n + 1, EMB)
    for l in range(2):
        msg[l] = _attention(w, embeds, l)
    hs = F.normalize(msg[:, :n, :], p=2, dim=2)
    ys = F.normalize(msg[:, n:, :], p=2, dim=2)
    aux_t = torch.as_tensor(np.asarray(aux, dtype=np.float32)).reshape(1, 2, 4)
    rep_row = torch.arange(n, dtype=torch.long)
    rep_col = torch.zeros(n, dtype=torch.long)
    q_list, w_layer = [], []
    for l in range(2):
        rep_y = spmm(rep_row, rep_col, ones_n, n, ys[l])
        outer = torch.matmul(torch.unsqueeze(hs[l], dim=2), torch.unsqueeze(rep_y, dim=1))
        cp = torch.reshape(torch.tile(w.cross, [n, 1]), [n, EMB, 1])
        emb = torch.reshape(torch.matmul(outer, cp), (n, EMB))
        hidden = torch.relu(torch.matmul(emb, w.h1))
        rep_aux = spmm(rep_row, rep_col, ones_n, n, aux_t[:, l, :])
        q_list.append(torch.matmul(torch.concat([hidden, rep_aux], 1), w.last_w))
        w_layer.append(torch.relu(rep_y @ w.wl1) @ w.wl2)
    mix = F.softmax(torch.concat(w_layer, dim=1), dim=1)
    q = mix[:, 0].unsqueeze(1) * q_list[0] + mix[:, 1].unsqueeze(1) * q_list[1]
    return q[:, 0].detach().numpy().copy()
