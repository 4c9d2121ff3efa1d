"""Host overhead per bench step of the single-graph headline (GMM N=1000 seed 0): wall time of
Engine.reset() and Engine.rollout() against the device time of their launches (HIP events),
medians over K steps, and the raw C-ABI md_rollout call alone (no Python array handling)."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine, gmm
K = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
eng.load_graphs([(1000,) + gmm.gmm_pair(1000, seed=0)])
for _ in range(3):
    eng.reset(); eng.rollout()
rw, rk, ow, ok, cw = [], [], [], [], []
tot = int(eng.node_off[-1])
seq = np.empty(tot, np.int32); lm = np.empty(tot, np.int32); ln = np.zeros(1, np.int32)
for _ in range(K):
    t0 = time.perf_counter(); eng.reset(); t1 = time.perf_counter()
    rk.append(eng.last_timing()[0]); rw.append((t1 - t0) * 1e3)
    t0 = time.perf_counter(); eng.rollout(); t1 = time.perf_counter()
    ok.append(eng.last_timing()[0]); ow.append((t1 - t0) * 1e3)
    eng.reset()
    t0 = time.perf_counter()
    st = eng.lib.md_rollout(eng.h, 1, seq.ctypes.data_as(_lib._i32p), lm.ctypes.data_as(_lib._i32p),
                            ln.ctypes.data_as(_lib._i32p), eng._ccb, None)
    cw.append((time.perf_counter() - t0) * 1e3 - eng.last_timing()[0])
m = lambda a: float(np.median(a))
print(f"reset: wall {m(rw):.3f} ms, kernel {m(rk):.3f} ms -> host {m(rw) - m(rk):.3f} ms")
print(f"rollout: wall {m(ow):.3f} ms, kernel {m(ok):.3f} ms -> host {m(ow) - m(ok):.3f} ms; raw md_rollout host {m(cw):.3f} ms")
print(f"step: wall {m(rw) + m(ow):.3f} ms, host {m(rw) - m(rk) + m(ow) - m(ok):.3f} ms")
