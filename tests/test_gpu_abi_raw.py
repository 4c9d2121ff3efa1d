"""The raw ctypes binding of INTEGRATION.md §2 (what a maintainer adds to the reference),
exercised end to end on the er100 golden graph: same sequence and AUDC as the reference."""
import ctypes

import numpy as np
import pytest

from conftest import load_golden
from mdcommunity_amd import _lib, engine

pytestmark = pytest.mark.gpu


def test_integration_snippet_er100():
    z = load_golden("er100")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    i32p = ctypes.POINTER(ctypes.c_int32)
    i64p = ctypes.POINTER(ctypes.c_int64)
    f32p = ctypes.POINTER(ctypes.c_float)
    SELECT_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, i32p)
    lib.md_create.argtypes = [ctypes.c_int, f32p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.md_load_graphs.argtypes = [ctypes.c_void_p, ctypes.c_int, i32p, i64p, i32p, i64p, i32p, f32p]
    lib.md_reset.argtypes = [ctypes.c_void_p, i32p]
    lib.md_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int, i32p, i32p, i32p, SELECT_CB, ctypes.c_void_p]
    lib.md_destroy.argtypes = [ctypes.c_void_p]
    lib.md_last_error.restype = ctypes.c_char_p

    def P(a, t):
        return a.ctypes.data_as(t)

    w = np.ascontiguousarray(engine.load_weights(engine.DEFAULT_UNIT), np.float32)
    ctx = ctypes.c_void_p()
    assert lib.md_create(0, P(w, f32p), w.size, 0, ctypes.byref(ctx)) == 0
    n = np.array([int(z["n_nodes"])], np.int32)
    e0 = np.ascontiguousarray(z["edges0"], np.int32)
    e1 = np.ascontiguousarray(z["edges1"], np.int32)
    o0 = np.array([0, len(e0)], np.int64)
    o1 = np.array([0, len(e1)], np.int64)
    assert lib.md_load_graphs(ctx, 1, P(n, i32p), P(o0, i64p), P(e0, i32p), P(o1, i64p), P(e1, i32p), None) == 0
    max_rank = np.zeros(1, np.int32)
    assert lib.md_reset(ctx, P(max_rank, i32p)) == 0

    @SELECT_CB
    def pick(user, graph, q, n_nodes, n_out, out):
        row = np.ctypeslib.as_array(q, shape=(n_nodes,))
        np.ctypeslib.as_array(out, shape=(n_out,))[:] = np.argsort(-row)[:n_out]
        return 0

    seq = np.zeros(n[0], np.int32)
    lmcc = np.zeros(n[0], np.int32)
    k = np.zeros(1, np.int32)
    assert lib.md_rollout(ctx, 1, P(seq, i32p), P(lmcc, i32p), P(k, i32p), pick, None) == 0, lib.md_last_error(ctx)
    score = 0.0
    for r in lmcc[:k[0]]:
        score += -1 * (-float(r) / (max_rank[0] * float(n[0])))
    lib.md_destroy(ctx)
    assert seq[:k[0]].tolist() == z["seq"].tolist()
    assert score == float(z["score"])
