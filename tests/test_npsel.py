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


def _endgame_picks(live, partner, value):
    """The per-step protocol of a K2 end-game: rows with every live node at `value`, the rest
    masked; np.argsort(-q)[0] picks, the pick and its partner leave (md_abi.cpp serve_endgame)."""
    live = live.copy()
    picks = []
    while live.any():
        q = np.where(live, value, MASK)
        a = int(np.argsort(-q)[0])
        assert live[a]
        picks.append(a)
        live[a] = live[partner[a]] = False
    return picks


def test_endgame_picks_depend_only_on_the_live_set():
    """The K2 end-game hand-shake runs every remaining pick on rows whose live entries hold one
    common value instead of the device's per-step Q: np.argsort(-q)[0] must not depend on that
    value (comparisons only), for any pairing and live set (the device ties all live nodes there,
    DESIGN.md)."""
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(4, 1200))
        npairs = int(rng.integers(1, n // 2 + 1))
        nodes = rng.permutation(n)[: 2 * npairs]
        partner = np.full(n, -1)
        partner[nodes[0::2]] = nodes[1::2]
        partner[nodes[1::2]] = nodes[0::2]
        live = partner >= 0
        ref = _endgame_picks(live, partner, -0.5)
        for v in (-0.0871, -0.0026, -3.0e-8, 0.25):
            assert _endgame_picks(live, partner, v) == ref
