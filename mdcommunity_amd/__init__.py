"""mdcommunity_amd — MI355X-native MultiDismantler inference rollout (gfx950 HIP kernels).

Drop-in for the reference's rollout path (KelvinRyman/MDCommunity,
``code/MultiDismantler_unit_cost``): the agent/env/graph classes mirror
``MultiDismantler_torch.py``, ``mvc_env.py`` and ``graph.py``; the per-step work runs in
``libmdroll.so`` (``include/mdroll.h``).
"""
__version__ = "0.1.0"
