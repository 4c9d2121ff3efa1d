"""Torn speculative slot, deterministically.

The iteration-1 prebuild of a single-graph dataflow rollout reads a speculative workgroup's
result slot (rows, kill list, degrees) before phase A confirms that result.  The diagnostic
build `make -C mdcommunity_amd/csrc torn-slot` (MD_TORN_SLOT + MD_DEBUG_BOUNDS) feeds every
third step's prebuild a torn slot: the degree words of odd nodes read as 0 (a half-rewritten
degree array, so nodes of degree 0 under any dmax, dmax = 1 included), the kill list's count
read as 0 (a stale kill list), and an early word naming the other slot of the pair (a slot is
rewritten only for a later request, which phase A of this step does not take).  The [1, dmax]
clamp of the first-layer row reads is compiled out and replaced by a counted check (sites 22 /
23, the reads it covered); every other index check raises an error.

Checked on gmm1000_s0 (one rollout, in a child process: the build is another library):
* no error -- no out-of-range access other than the clamp-covered row reads, which the check
  blocked and counted (> 0: the injection reached them);
* in every torn step with a forward pass, tiles ran without the confirmed prebuild (the
  confirmation discarded it);
* the rollout equals the certified sequence, the LMCC trace the reference's, AUDC bit-exact.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import load_golden
from test_certificates import load_cert

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TORN = os.path.join(ROOT, "mdcommunity_amd", "csrc", "build", "libmdroll_torn.so")
CAP = 512
CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from mdcommunity_amd import _lib, engine
z = np.load(sys.argv[2])
cap = int(sys.argv[3])
e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
try:
    e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
    mr = int(e.reset()[0])
    e.profile(cap)
    err = None
    try:
        seq, ranks = e.rollout()[0]
    except Exception as ex:  # an index check other than the counted ones
        err, seq, ranks = str(ex), np.zeros(0, np.int32), np.zeros(0, np.int32)
    P = e.profile_read(cap).astype(np.int64)
    e.profile(0)
finally:
    e.close()
fwd = [int(t) for t in range(min(len(seq), len(P))) if P[t, 10] > 0]
print(json.dumps({"err": err, "seq": seq.tolist(), "ranks": ranks.tolist(), "max_rank": mr,
                  "blocked": [int(P[0, 92]), int(P[0, 93])],
                  "no_prebuild": {str(t): int(P[t, 79]) for t in fwd},
                  "pre_state": {str(t): int(P[t, 78]) for t in fwd}}))
"""


def test_torn_slot_prebuild_discarded_in_bounds():
    if not os.path.exists(TORN):
        pytest.skip("diagnostic build missing: make -C mdcommunity_amd/csrc torn-slot")
    name = "gmm1000_s0"
    z, c = load_golden(name), load_cert(name)
    from conftest import GOLDEN
    env = dict(os.environ, MD_LIB=TORN)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, os.path.join(GOLDEN, f"rollout_{name}.npz"), str(CAP)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["err"] is None, res["err"]
    # the injected degree-0 / out-of-table rows reached the reads the clamp covered, blocked there
    assert sum(res["blocked"]) > 0, (res["blocked"], res["pre_state"], res["no_prebuild"])
    # every torn step with a forward pass: its prebuild was not confirmed (tiles rebuilt)
    torn = {int(t): k for t, k in res["no_prebuild"].items() if int(t) % 3 == 1}
    assert torn and all(k > 0 for k in torn.values()), torn
    # and the rollout is the certified one
    n, mr = int(z["n_nodes"]), res["max_rank"]
    assert res["seq"] == c["gpu_seq"].tolist()
    assert res["ranks"] == c["ref_ranks_along"].tolist()
    s = 0.0
    for x in res["ranks"]:
        s += -1 * (-float(x) / (mr * float(n)))
    assert s == float(z["score"])
