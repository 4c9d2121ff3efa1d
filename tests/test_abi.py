"""The C-ABI library builds, loads and exports every symbol include/mdroll.h declares.
No compute calls here (no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from mdcommunity_amd import _lib

HEADER = os.path.join(ROOT, "include", "mdroll.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:md_status|void|int|const char\*)\s+(md_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "mdcommunity_amd", "csrc")], check=True)
    return _lib.load_library()


def test_exports_match_header(lib):
    syms = header_symbols()
    assert len(syms) >= 15
    assert sorted(_lib.EXPORTS) == syms
    for s in syms:
        assert hasattr(lib, s), s


def test_version_and_no_gpu_errors(lib):
    assert b"gfx950" in lib.md_version()
    w = np.zeros(_lib.MD_WEIGHT_FLOATS, np.float32)
    h = ctypes.c_void_p()
    bad = lib.md_create(0, w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 5, 0, ctypes.byref(h))
    assert bad == _lib.MD_EINVAL  # wrong weight count is rejected before any HIP call
    assert lib.md_reset(None, None) == _lib.MD_EINVAL
    assert lib.md_last_error(None) == b"null context"
    assert lib.md_device_count() == 0  # no GPU in the build container


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_weight_packing_order():
    """pack_weights follows the MD_WEIGHT_FLOATS layout documented in mdroll.h."""
    from mdcommunity_amd import engine
    st = engine.load_state(engine.DEFAULT_UNIT)
    w = _lib.pack_weights(st)
    assert w.size == 31205
    assert np.array_equal(w[128:128 + 4096].reshape(64, 64), st["p_node_conv"])
    assert np.array_equal(w[18560:18596], st["h2_weight"].reshape(-1))
    assert np.array_equal(w[26980:26980 + 4096].reshape(64, 64), st["layerNodeAttention_weight.trans"])
    assert w[31204] == st["layerNodeAttention_weight.logis.parameter.bias"][0]
