"""Host-side helpers around the device engine: weight files and shared contexts."""
import os

import numpy as np

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
WEIGHTS_DIR = os.path.join(HERE, "weights")

# Reference checkpoint paths (relative to the variant directory, as the scripts name them)
# -> (variant, the fp32 arrays converted from them by scripts/convert_ckpt.py, cost mode).
KNOWN_CKPTS = {
    ("MultiDismantler_unit_cost", "models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt"):
        ("unit_g0.5_iter100000.npz", _lib.MD_COST_UNIT),        # U/testSynthetic.py:19
    ("MultiDismantler_unit_cost", "models/g0-1_10w_TORCH-Model_GMM_30_50/nrange_30_50_iter_24000.ckpt"):
        ("unit_g0-1_iter24000.npz", _lib.MD_COST_UNIT),         # U/testReal.py:78-79,100
    ("MultiDismantler_degree_cost", "models/nrange_30_50_iter_100000.ckpt"):
        ("degree_iter100000.npz", _lib.MD_COST_DEGREE),         # D/testReal.py:53,79
}
VARIANT_DIRS = ("MultiDismantler_unit_cost", "MultiDismantler_degree_cost", "CEMultiDismantler", "HCA-Dismantler")
DEFAULT_UNIT = os.path.join(WEIGHTS_DIR, "unit_g0.5_iter100000.npz")
DEFAULT_UNIT_REAL = os.path.join(WEIGHTS_DIR, "unit_g0-1_iter24000.npz")
DEFAULT_DEGREE = os.path.join(WEIGHTS_DIR, "degree_iter100000.npz")
SHIPPED_COST = {npz: cost for npz, cost in KNOWN_CKPTS.values()}


def resolve_model(path, cost_mode=None):
    """Map a reference checkpoint path to a loadable file.

    An existing file is returned as is.  Otherwise the path must name one of the reference's
    own checkpoints by its variant-relative path (``./models/...`` as the scripts write it,
    optionally under its variant directory); the shipped .npz converted from it is returned.
    With ``cost_mode`` given, a shipped checkpoint of the other cost model is refused (the
    unit-cost agent must not silently run degree-cost weights, or the reverse).  Anything
    else raises FileNotFoundError.
    """
    if path is None:
        return DEFAULT_DEGREE if cost_mode == _lib.MD_COST_DEGREE else DEFAULT_UNIT
    if os.path.exists(path):
        shipped = SHIPPED_COST.get(os.path.basename(path))
        if (shipped is not None and cost_mode is not None and shipped != cost_mode
                and os.path.dirname(os.path.abspath(path)) == WEIGHTS_DIR):
            raise ValueError(f"{path} holds {'degree' if shipped else 'unit'}-cost weights; this agent is "
                             f"{'degree' if cost_mode else 'unit'} cost")
        return path
    norm = os.path.normpath(path.replace("\\", "/")).replace("\\", "/")
    parts = norm.split("/")
    variant = next((d for d in parts if d in VARIANT_DIRS), None)
    for (var, key), (npz, cost) in KNOWN_CKPTS.items():
        if not (norm == key or norm.endswith("/" + key)):
            continue
        if variant is not None and variant != var:
            continue
        if cost_mode is not None and cost != cost_mode:
            raise ValueError(f"{path} is a {'degree' if cost else 'unit'}-cost checkpoint "
                             f"({var}); this agent is {'degree' if cost_mode else 'unit'} cost")
        return os.path.join(WEIGHTS_DIR, npz)
    raise FileNotFoundError(f"{path}: not a file, and not one of the reference's checkpoints "
                            f"({', '.join(k for _, k in KNOWN_CKPTS)})")


def load_state(path, cost_mode=None):
    """state_dict arrays of a model file: .npz (ours) or a reference .ckpt loaded with
    torch.load(weights_only=True) (U/MultiDismantler_torch.py:791-797)."""
    path = resolve_model(path, cost_mode)
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    import torch
    sd = torch.load(path, weights_only=True, map_location="cpu")
    return {k: v.detach().cpu().numpy() for k, v in sd.items()}


def load_weights(path, cost_mode=None):
    return _lib.pack_weights(load_state(path, cost_mode))


_mcc_engine = None


def initial_lmcc(g):
    """Graph_test.max_rank (U/graph.py:80-84) computed by the device MCC (md_reset)."""
    global _mcc_engine
    if _mcc_engine is None:
        _mcc_engine = _lib.Engine(np.zeros(_lib.MD_WEIGHT_FLOATS, np.float32))
    _mcc_engine.load_graphs([(g.num_nodes, g.edges[0], g.edges[1])])
    return int(_mcc_engine.reset()[0])
