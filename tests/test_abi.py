"""The C-ABI library loads and exports every symbol include/krrn_hip.h declares, and rejects bad
arguments with the documented codes on the host side (no GPU needed: the checks run before any
HIP call)."""
import ctypes
import os
import re

import pytest

from pose_estimation_amd import _lib
from pose_estimation_amd import bpnp, dataset, fps, loss, metric, runtime  # noqa: F401  (register the signatures)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "krrn_hip.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^int (krrn_\w+)\(", src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert len(names) >= 15
    assert "krrn_conv2d_f32" in names and "krrn_pnp_ransac_f32" in names


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    for name in _declared():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"


def test_ctypes_signatures_match_header_arity():
    src = open(HEADER).read()
    for name in _declared():
        m = re.search(rf"^int {name}\((.*?)\);", src, re.M | re.S)
        nargs = len([a for a in m.group(1).split(",") if a.strip()])
        assert nargs == len(_lib.SIGNATURES[name]), (name, nargs, len(_lib.SIGNATURES[name]))


def test_host_side_errors():
    lib = _lib.lib()
    N = ctypes.c_void_p(0)
    # null pointers -> KRRN_EARG
    assert lib.krrn_knn_f32(N, 0, 3, 10, N, N, 0, 3, 10, 3, 4, 1, 0, 1, N, N) == -1
    fake = ctypes.c_void_p(16)
    # d must be 3 or 9 -> KRRN_ESHAPE
    assert lib.krrn_knn_f32(fake, 0, 3, 10, N, fake, 0, 3, 10, 4, 4, 1, 0, 1, fake, N) == -2
    # k + drop > 16 -> KRRN_ESHAPE
    assert lib.krrn_knn_f32(fake, 0, 3, 10, N, fake, 0, 3, 100, 3, 16, 1, 0, 1, fake, N) == -2
    # conv: cin not a multiple of 4 -> KRRN_EALIGN
    taps = (ctypes.c_int * 9)()
    assert lib.krrn_conv2d_f32(fake, 4, 0, 1, 8, 8, 3, 8, 8, 1, 1, taps, taps, fake, 4, 4, N, N, N, 1, N, 0, 0,
                               fake, 4, 0, 8, 8, 1, 1, 0, 0, 0, 0, 0, 1, N, N) == -3
    # pnp: P < 5 -> KRRN_ESHAPE
    assert lib.krrn_pnp_ransac_f32(fake, 16, fake, 10, fake, 4, fake, fake, fake, fake, fake, fake, 10,
                                   ctypes.c_float(1.0), ctypes.c_double(0.9999), fake, fake, fake, fake, N, 1, N) == -2
    # NCHW 1x1 split form: null weights -> KRRN_EARG; N outside (32, 80] or cin != 128 -> KRRN_ESHAPE;
    # misaligned channel offset -> KRRN_EALIGN
    nchw_x3 = lib.krrn_conv1x1_nchw_x3_f32
    assert nchw_x3(fake, 128, 0, 1, 64, 128, N, 72, 72, N, N, fake, 72, 0, N) == -1
    assert nchw_x3(fake, 128, 0, 1, 64, 128, fake, 16, 16, N, N, fake, 16, 0, N) == -2
    assert nchw_x3(fake, 256, 0, 1, 64, 256, fake, 72, 72, N, N, fake, 72, 0, N) == -2
    assert nchw_x3(fake, 136, 2, 1, 64, 128, fake, 72, 72, N, N, fake, 72, 0, N) == -3
    with pytest.raises(RuntimeError, match="KRRN_EARG"):
        _lib.check(-1, "x")
