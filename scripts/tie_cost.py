"""Per-step device time of the headline rollout split by whether the step's prediction was an
exact tie (host hand-shake) -- gmm1000_s0, dedicated mode, workgroup-0 phase stamps."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine

z = np.load(os.path.join(ROOT, "tests/golden/rollout_gmm1000_s0.npz"))
eng = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
eng.load_graphs([(1000, z["edges0"], z["edges1"])])
eng.reset(); eng.rollout()
eng.reset(); eng.profile(512); eng.rollout()
P = eng.profile_read().astype(np.int64)
eng.profile(0)
tr = eng.trace(0)
full = P[P[:, 10] > 0]
stp = (full[:, 10] - full[:, 0]) / 100.0
A = (full[:, 3] - full[:, 0]) / 100.0
ties = np.asarray(tr["n_tie"])[: len(stp)] > 1
print("steps %d, ties %d" % (len(stp), int(ties.sum())))
print("non-tie steps: mean %.1f us (phase A %.1f); tie steps: mean %.1f us (phase A %.1f)" % (
    stp[~ties].mean(), A[~ties].mean(), stp[ties].mean(), A[ties].mean()))
print("n_live at tie steps:", np.asarray(tr["n_live"])[: len(stp)][ties].tolist())
print("tie step times:", np.round(stp[ties], 1).tolist())
print("tie phase A:", np.round(A[ties], 1).tolist())
