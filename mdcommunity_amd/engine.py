"""Host-side helpers around the device engine: weight files and shared contexts."""
import os

import numpy as np

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
WEIGHTS_DIR = os.path.join(HERE, "weights")

# Reference checkpoint paths (relative to the variant directory, as the scripts name them)
# -> the fp32 arrays converted from them by scripts/convert_ckpt.py.
KNOWN_CKPTS = {
    "g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt": "unit_g0.5_iter100000.npz",   # U/testSynthetic.py:19
    "g0-1_10w_TORCH-Model_GMM_30_50/nrange_30_50_iter_24000.ckpt": "unit_g0-1_iter24000.npz",  # U/testReal.py:150
    "nrange_30_50_iter_100000.ckpt": "degree_iter100000.npz",                                  # D/testReal.py:79
}
DEFAULT_UNIT = os.path.join(WEIGHTS_DIR, "unit_g0.5_iter100000.npz")
DEFAULT_UNIT_REAL = os.path.join(WEIGHTS_DIR, "unit_g0-1_iter24000.npz")
DEFAULT_DEGREE = os.path.join(WEIGHTS_DIR, "degree_iter100000.npz")


def resolve_model(path):
    """Map a reference checkpoint path to a loadable file (the shipped .npz when the
    reference's models/ directory is not present)."""
    if path is None:
        return DEFAULT_UNIT
    if os.path.exists(path):
        return path
    norm = path.replace("\\", "/")
    for key, npz in KNOWN_CKPTS.items():
        if norm.endswith(key):
            return os.path.join(WEIGHTS_DIR, npz)
    raise FileNotFoundError(path)


def load_state(path):
    """state_dict arrays of a model file: .npz (ours) or a reference .ckpt loaded with
    torch.load(weights_only=True) (U/MultiDismantler_torch.py:791-797)."""
    path = resolve_model(path)
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    import torch
    sd = torch.load(path, weights_only=True, map_location="cpu")
    return {k: v.detach().cpu().numpy() for k, v in sd.items()}


def load_weights(path):
    return _lib.pack_weights(load_state(path))


_mcc_engine = None


def initial_lmcc(g):
    """Graph_test.max_rank (U/graph.py:80-84) computed by the device MCC (md_reset)."""
    global _mcc_engine
    if _mcc_engine is None:
        _mcc_engine = _lib.Engine(np.zeros(_lib.MD_WEIGHT_FLOATS, np.float32))
    _mcc_engine.load_graphs([(g.num_nodes, g.edges[0], g.edges[1])])
    return int(_mcc_engine.reset()[0])
