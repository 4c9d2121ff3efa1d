#!/usr/bin/env python3
"""Convert the reference's torch ``state_dict`` checkpoints into plain ``.npz`` weight files.

The reference loads checkpoints with ``torch.load`` (``U/MultiDismantler_torch.py:791-797``).
``/root/reference`` does not exist on the GPU box, so the three checkpoints the rollout
scripts use are converted once, here, with the safe loader (``weights_only=True``) and the
resulting fp32 arrays are committed under ``mdcommunity_amd/weights/``:

* ``unit_g0.5_iter100000.npz``  <- ``U/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt``
  (``U/testSynthetic.py:19``)
* ``unit_g0-1_iter24000.npz``   <- ``U/models/g0-1_10w_TORCH-Model_GMM_30_50/nrange_30_50_iter_24000.ckpt``
  (``U/testReal.py:150``)
* ``degree_iter100000.npz``     <- ``D/models/nrange_30_50_iter_100000.ckpt`` (``D/testReal.py:79``)

Only data moves; no reference code is copied.
"""
import os
import sys

import numpy as np
import torch

REF = "/root/reference/code"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mdcommunity_amd", "weights")

CKPTS = {
    "unit_g0.5_iter100000.npz":
        "MultiDismantler_unit_cost/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt",
    "unit_g0-1_iter24000.npz":
        "MultiDismantler_unit_cost/models/g0-1_10w_TORCH-Model_GMM_30_50/nrange_30_50_iter_24000.ckpt",
    "degree_iter100000.npz":
        "MultiDismantler_degree_cost/models/nrange_30_50_iter_100000.ckpt",
}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, rel in CKPTS.items():
        sd = torch.load(os.path.join(REF, rel), weights_only=True, map_location="cpu")
        arrs = {k: v.detach().cpu().numpy().astype(np.float32) for k, v in sd.items()}
        np.savez(os.path.join(OUT, name), **arrs)
        print(name, sum(a.size for k, a in arrs.items() if k != "last_w"), "params")
    return 0


if __name__ == "__main__":
    sys.exit(main())
