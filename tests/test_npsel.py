"""The tie hand-shake's native selection: numpy's own float64 argsort routine, reached through
the _npsel helper, must order exactly like np.argsort(-q) (the reference's rule,
U/MultiDismantler_torch.py:725,769) -- checked on tie-heavy masked rows, no GPU needed."""
import ctypes

import numpy as np
import pytest

_npsel = pytest.importorskip("mdcommunity_amd._npsel")
MASK = -1073741823.5  # U/MultiDismantler_torch.py:60
ARGSORT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)


def test_native_argsort_equals_numpy_on_ties():
    fn = ARGSORT(_npsel.argsort_f64())
    rng = np.random.default_rng(7)
    for _ in range(1500):
        n = int(rng.integers(2, 1300))
        q = rng.integers(0, max(2, n // int(rng.integers(1, 60))), size=n).astype(np.float64) * 0.013
        q[rng.random(n) < rng.random()] = MASK
        neg = np.ascontiguousarray(-q)
        idx = np.arange(n, dtype=np.int64)
        assert fn(neg.ctypes.data, idx.ctypes.data, n, None) >= 0
        assert np.array_equal(idx, np.argsort(-q))
