"""CPU oracle for the MultiDismantler inference rollout — TEST INFRASTRUCTURE ONLY.

This package restates, on the host CPU, the reference algorithm of the hot path
(KelvinRyman/MDCommunity, ``code/MultiDismantler_unit_cost`` = ``U/``):

* ``oracle.refmodel``  the Q network forward, op for op in torch-CPU
  (``U/MultiDismantler_net_graphsage.py:243-394``, ``U/MRGNN/mutil_layer_weight.py:252-313``);
* ``oracle.refenv``    featurisation (``U/PrepareBatchGraph.py:35-177``), environment and
  mutual-LMCC cascade (``U/mvc_env.py:31-137``, ``U/Mcc.py:3-38``) and the rollout loop
  (``U/MultiDismantler_torch.py:263-302,711-784``).

Pinning: the restatement is checked against golden vectors produced by running the
reference itself in the build container (``tests/golden/make_golden.py``): removal
sequences, LMCC traces and AUDC bit-exact, and Q rows bit-exact on the build host.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker or as the timed CPU baseline.  The product
path (``mdcommunity_amd``) never imports it.
"""
