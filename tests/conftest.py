import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libmdroll.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


MASK = -(2147483647 / 2)  # U/MultiDismantler_torch.py:60


def load_golden(name):
    """A rollout fixture as a dict.  The reference's masked Q row of every prediction is stored
    as float32 with NaN at the mask (``q_all``, lossless); it is handed out as the float64
    rows the reference's Predict returns (``q_rows``, mask -1073741823.5) with ``q_steps``."""
    import numpy as np
    with np.load(os.path.join(GOLDEN, f"rollout_{name}.npz")) as z:
        d = {k: z[k] for k in z.files}
    if "q_all" in d:
        q = d["q_all"].astype(np.float64)
        d["q_rows"] = np.where(np.isnan(q), MASK, q)
        d["q_steps"] = np.arange(len(q), dtype=np.int32)
    return d
