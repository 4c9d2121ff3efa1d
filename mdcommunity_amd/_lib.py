"""ctypes binding of ``libmdroll.so`` (the C ABI in ``include/mdroll.h``).

The shared library is built in-tree (``mdcommunity_amd/libmdroll.so``) by
``__graft_entry__.build()`` or ``make -C mdcommunity_amd/csrc``.  There is no fallback:
if the library or a GPU is missing, every entry point raises.
"""
import ctypes
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MD_LIB overrides the library path (A/B comparisons of builds on the GPU box)
LIB_PATH = os.environ.get("MD_LIB") or os.path.join(HERE, "libmdroll.so")

MD_OK, MD_EINVAL, MD_EHIP, MD_EOOM, MD_ESTATE, MD_ETIMEOUT, MD_ECALLBACK = range(7)
MD_COST_UNIT, MD_COST_DEGREE = 0, 1
MD_WEIGHT_FLOATS = 31205
STATUS_NAMES = {1: "MD_EINVAL", 2: "MD_EHIP", 3: "MD_EOOM", 4: "MD_ESTATE", 5: "MD_ETIMEOUT", 6: "MD_ECALLBACK"}

# Every symbol include/mdroll.h declares (checked by tests/test_abi.py).
PROF_SLOTS = 96  # MD_PROF_SLOTS in include/mdroll.h

EXPORTS = ("md_create", "md_destroy", "md_last_error", "md_set_weights", "md_load_graphs", "md_reset",
           "md_reset_deferred", "md_max_rank",
           "md_predict", "md_step", "md_rollout", "md_rollout_packed", "md_rollout_trace", "md_get_state", "md_set_state",
           "md_set_team_size", "md_set_tie_argsort", "md_last_timing", "md_host_requests", "md_profile", "md_profile_read",
           "md_version", "md_device_count", "md_spec_stats", "md_gmm_last_error", "md_gmm_nodes", "md_gmm_links")

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
SELECT_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, _f64p, ctypes.c_int, ctypes.c_int, _i32p)
# the same C type with the row and the output as plain addresses (cheaper to receive: the
# engine's callback wraps each host buffer as an ndarray once and reuses the view)
SELECT_CB_ADDR = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_void_p)

_lib = None


class MDError(RuntimeError):
    pass


def load_library(path=LIB_PATH):
    """Load and prototype libmdroll.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MDError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                      "or `make -C mdcommunity_amd/csrc` (hipcc, gfx950)")
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    proto = {
        "md_create": (ctypes.c_int, [ctypes.c_int, _f32p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(vp)]),
        "md_destroy": (None, [vp]),
        "md_last_error": (ctypes.c_char_p, [vp]),
        "md_set_weights": (ctypes.c_int, [vp, _f32p, ctypes.c_size_t]),
        "md_load_graphs": (ctypes.c_int, [vp, ctypes.c_int, _i32p, _i64p, _i32p, _i64p, _i32p, _f32p]),
        "md_reset": (ctypes.c_int, [vp, _i32p]),
        "md_reset_deferred": (ctypes.c_int, [vp]),
        "md_max_rank": (ctypes.c_int, [vp, _i32p]),
        "md_predict": (ctypes.c_int, [vp, _f32p, _i32p, _i32p, _f32p]),
        "md_step": (ctypes.c_int, [vp, _i32p, _i32p, _u8p]),
        "md_rollout": (ctypes.c_int, [vp, ctypes.c_int, _i32p, _i32p, _i32p, SELECT_CB_ADDR, vp]),
        "md_rollout_packed": (ctypes.c_int, [vp, ctypes.c_int, _i32p, _i32p, _i32p, SELECT_CB_ADDR, vp]),
        "md_rollout_trace": (ctypes.c_int, [vp, ctypes.c_int, _i32p, _i32p, _i32p, _i32p, _f32p, _f32p, _i32p]),
        "md_spec_stats": (ctypes.c_int, [vp, ctypes.c_int, _i32p, _i32p]),
        "md_get_state": (ctypes.c_int, [vp, ctypes.c_int, _u8p, _u8p, _u8p, _i32p]),
        "md_set_state": (ctypes.c_int, [vp, ctypes.c_int, _u8p, _u8p, _u8p]),
        "md_set_team_size": (ctypes.c_int, [vp, ctypes.c_int]),
        "md_set_tie_argsort": (ctypes.c_int, [vp, vp]),
        "md_last_timing": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), _i32p]),
        "md_host_requests": (ctypes.c_int, [vp, _i32p]),
        "md_profile": (ctypes.c_int, [vp, ctypes.c_int]),
        "md_profile_read": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, _i32p]),
        "md_version": (ctypes.c_char_p, []),
        "md_device_count": (ctypes.c_int, []),
        "md_gmm_last_error": (ctypes.c_char_p, []),
        "md_gmm_nodes": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), _f64p,
                                        _f64p, _f64p, _f64p, _f64p]),
        "md_gmm_links": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p, _f64p, _f64p, _f64p,
                                        ctypes.POINTER(ctypes.c_uint64), _i32p, _i64p, ctypes.c_int64, _i64p, _i64p,
                                        ctypes.c_int64]),
    }
    for name, (res, args) in proto.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def device_count():
    """Visible GPUs (md_device_count; 0 without a GPU or when the runtime fails)."""
    return int(load_library().md_device_count())


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


_NPSEL = []


def _numpy_argsort_ptr():
    """Address of numpy's own float64 argsort routine (the one np.argsort runs), from the
    package's _npsel helper; None when the helper is not built (the Python callback is used)."""
    if not _NPSEL:
        try:
            from . import _npsel
            _NPSEL.append(_npsel.argsort_f64())
        except ImportError:
            _NPSEL.append(None)
    return _NPSEL[0]


def _argsort_select(q, n_out):
    """The reference's selection rule: ``np.argsort(-q)[:step]`` on the masked float64 row
    (U/MultiDismantler_torch.py:725,769)."""
    return np.argsort(-q)[:n_out]


class Engine:
    """One device context (md_ctx) holding weights and a batch of graphs."""

    def __init__(self, weights, device=0, cost_mode=MD_COST_UNIT):
        self.lib = load_library()
        w = np.ascontiguousarray(weights, dtype=np.float32).reshape(-1)
        if w.size != MD_WEIGHT_FLOATS:
            raise ValueError(f"expected {MD_WEIGHT_FLOATS} packed weights, got {w.size}")
        self.cost_mode = cost_mode
        h = ctypes.c_void_p()
        self._check(self.lib.md_create(device, _ptr(w, _f32p), w.size, cost_mode, ctypes.byref(h)), None)
        self.h = h
        self.n_nodes = None
        self.node_off = None
        self._cb_error = None
        self.selector = _argsort_select
        self._tie_native = False  # the argsort routine registered with md_set_tie_argsort (False: none yet)
        self._views = {}
        wr = weakref.ref(self)  # no reference cycle through the thunk: close() still runs from __del__

        def cb(user, g, qp, n, n_out, out):
            eng = wr()
            return eng._select_cb(user, g, qp, n, n_out, out) if eng is not None else 1

        self._ccb = SELECT_CB_ADDR(cb)  # one C thunk per engine (the hot path reuses it)

    def _check(self, st, h="self"):
        if st != MD_OK:
            handle = self.h if h == "self" else h
            msg = self.lib.md_last_error(handle).decode() if handle else ""
            raise MDError(f"{STATUS_NAMES.get(st, st)}: {msg}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.md_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_weights(self, weights):
        w = np.ascontiguousarray(weights, dtype=np.float32).reshape(-1)
        self._check(self.lib.md_set_weights(self.h, _ptr(w, _f32p), w.size))

    def set_team_size(self, t):
        self._check(self.lib.md_set_team_size(self.h, int(t)))

    def load_graphs(self, graphs, node_w=None):
        """graphs: list of (n, edges0 [E0,2], edges1 [E1,2]) in reference edge order."""
        n = np.asarray([int(g[0]) for g in graphs], dtype=np.int32)
        e = [[np.asarray(g[1 + l], dtype=np.int32).reshape(-1, 2) for g in graphs] for l in range(2)]
        offs = [np.concatenate([[0], np.cumsum([len(x) for x in e[l]])]).astype(np.int64) for l in range(2)]
        flat = [np.ascontiguousarray(np.concatenate(e[l]) if offs[l][-1] else np.zeros((1, 2), np.int32),
                                     dtype=np.int32) for l in range(2)]
        nw = None
        if node_w is not None:
            nw = np.ascontiguousarray(node_w, dtype=np.float32).reshape(-1)
        self._check(self.lib.md_load_graphs(self.h, len(graphs), _ptr(n, _i32p), _ptr(offs[0], _i64p),
                                            _ptr(flat[0], _i32p), _ptr(offs[1], _i64p), _ptr(flat[1], _i32p),
                                            _ptr(nw, _f32p)))
        self.n_nodes = n
        self.node_off = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
        self.n_edges = [np.diff(offs[l]) for l in range(2)]

    def reset(self):
        mr = np.zeros(len(self.n_nodes), np.int32)
        self._check(self.lib.md_reset(self.h, _ptr(mr, _i32p)))
        return mr

    def reset_deferred(self):
        """reset() with MvcEnv.s0's prune run as the first environment step of the next
        rollout() (one launch, no separate s0 launch); max_rank() after that rollout."""
        self._check(self.lib.md_reset_deferred(self.h))

    def max_rank(self):
        mr = np.zeros(len(self.n_nodes), np.int32)
        self._check(self.lib.md_max_rank(self.h, _ptr(mr, _i32p)))
        return mr

    def predict(self):
        q = np.zeros(int(self.node_off[-1]), np.float32)
        am = np.zeros(len(self.n_nodes), np.int32)
        nt = np.zeros(len(self.n_nodes), np.int32)
        gap = np.zeros(len(self.n_nodes), np.float32)
        self._check(self.lib.md_predict(self.h, _ptr(q, _f32p), _ptr(am, _i32p), _ptr(nt, _i32p), _ptr(gap, _f32p)))
        return q, am, nt, gap

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        lm = np.zeros(len(self.n_nodes), np.int32)
        term = np.zeros(len(self.n_nodes), np.uint8)
        self._check(self.lib.md_step(self.h, _ptr(a, _i32p), _ptr(lm, _i32p), _ptr(term, _u8p)))
        return lm, term.astype(bool)

    def _view(self, addr, n, ct, dt):
        key = (addr, n, dt)
        a = self._views.get(key)
        if a is None:
            a = self._views[key] = np.frombuffer((ct * n).from_address(addr), dtype=dt)
        return a

    def _select_cb(self, user, g, qp, n, n_out, out):
        # the row is the library's buffer, valid during the call (the selector must not keep
        # it); hot path of every tied step, hence the cached views
        try:
            q = self._view(qp, n, ctypes.c_double, np.float64)
            sel = self.selector(q, n_out)
            o = self._view(out, n_out, ctypes.c_int32, np.int32)
            o[:] = sel[:n_out]
            return 0
        except Exception as ex:  # surfaced after md_rollout returns
            self._cb_error = ex
            return 1

    def rollout(self, step=1):
        # the default rule np.argsort(-q)[:step] runs on the library's host thread through numpy's
        # own argsort routine; a custom selector goes through the callback
        native = _numpy_argsort_ptr() if self.selector is _argsort_select else None
        if native != self._tie_native:
            self._check(self.lib.md_set_tie_argsort(self.h, native))
            self._tie_native = native
        tot = int(self.node_off[-1])
        # packed outputs (md_rollout_packed): only the removals cross the link; each call's
        # arrays are fresh, so the per-graph views below are not shared with later calls
        seq = np.empty(tot, np.int32)
        lm = np.empty(tot, np.int32)
        ln = np.zeros(len(self.n_nodes), np.int32)
        self._cb_error = None
        st = self.lib.md_rollout_packed(self.h, int(step), _ptr(seq, _i32p), _ptr(lm, _i32p), _ptr(ln, _i32p),
                                        self._ccb, None)
        if self._cb_error is not None:
            raise self._cb_error
        self._check(st)
        ends = np.cumsum(ln).tolist()
        starts = [0] + ends[:-1]
        return [(seq[a:b], lm[a:b]) for a, b in zip(starts, ends)]

    def trace(self, g):
        n = int(self.n_nodes[g])
        arrs = [np.zeros(n, np.int32) for _ in range(4)]
        qm = np.zeros(n, np.float32)
        gp = np.zeros(n, np.float32)
        npred = ctypes.c_int32()
        self._check(self.lib.md_rollout_trace(self.h, g, *[_ptr(a, _i32p) for a in arrs], _ptr(qm, _f32p),
                                              _ptr(gp, _f32p), ctypes.byref(npred)))
        k = npred.value
        return dict(n_live=arrs[0][:k], m0=arrs[1][:k], m1=arrs[2][:k], n_tie=arrs[3][:k], qmax=qm[:k], gap=gp[:k])

    def spec_stats(self, g):
        """(removals whose fixed point came from a speculative workgroup, removals) of graph g
        in the last rollout (diagnostics; md_spec_stats)."""
        hits, rem = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.md_spec_stats(self.h, int(g), ctypes.byref(hits), ctypes.byref(rem)))
        return hits.value, rem.value

    def get_state(self, g):
        n = int(self.n_nodes[g])
        cov = np.zeros(n, np.uint8)
        r0 = np.zeros(max(1, int(self.n_edges[0][g])), np.uint8)
        r1 = np.zeros(max(1, int(self.n_edges[1][g])), np.uint8)
        cnt = np.zeros(6, np.int32)
        self._check(self.lib.md_get_state(self.h, g, _ptr(cov, _u8p), _ptr(r0, _u8p), _ptr(r1, _u8p), _ptr(cnt, _i32p)))
        return cov.astype(bool), r0[:int(self.n_edges[0][g])].astype(bool), r1[:int(self.n_edges[1][g])].astype(bool), cnt

    def set_state(self, g, covered, removed0, removed1):
        cov = np.ascontiguousarray(covered, dtype=np.uint8)
        r0 = np.ascontiguousarray(removed0, dtype=np.uint8)
        r1 = np.ascontiguousarray(removed1, dtype=np.uint8)
        self._check(self.lib.md_set_state(self.h, g, _ptr(cov, _u8p), _ptr(r0, _u8p), _ptr(r1, _u8p)))

    def profile(self, steps):
        self._check(self.lib.md_profile(self.h, int(steps)))

    def profile_read(self, cap=4096):
        out = np.zeros((cap, PROF_SLOTS), np.uint64)
        k = ctypes.c_int32()
        self._check(self.lib.md_profile_read(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap,
                                             ctypes.byref(k)))
        return out[:k.value]

    def host_requests(self):
        """Host selection requests served during the last call (ties, stepRatio predictions)."""
        n = ctypes.c_int32()
        self._check(self.lib.md_host_requests(self.h, ctypes.byref(n)))
        return n.value

    def last_timing(self):
        ms = ctypes.c_double()
        nl = ctypes.c_int32()
        self._check(self.lib.md_last_timing(self.h, ctypes.byref(ms), ctypes.byref(nl)))
        return ms.value, nl.value


def pack_weights(arrays):
    """Pack a reference state_dict (name -> array) into the MD_WEIGHT_FLOATS blob of mdroll.h."""
    order = ["w_n2l", "p_node_conv", "p_node_conv2", "p_node_conv3", "h1_weight", "h2_weight", "cross_product",
             "w_layer1", "w_layer2", "layerNodeAttention_weight.trans", "layerNodeAttention_weight.bias",
             "layerNodeAttention_weight.logis.parameter.weight", "layerNodeAttention_weight.logis.parameter.bias"]
    parts = []
    for k in order:
        a = arrays.get(k)
        if a is None and k == "h2_weight":
            a = arrays["last_w"]
        parts.append(np.asarray(a, dtype=np.float32).reshape(-1))
    w = np.concatenate(parts)
    assert w.size == MD_WEIGHT_FLOATS, w.size
    return w
