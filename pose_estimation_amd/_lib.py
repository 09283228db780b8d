"""Loader for the in-tree C-ABI library ``libkrrn_hip.so`` (include/krrn_hip.h).

The library is the product path: there is no CPU or PyTorch fallback. If it is
missing, ``lib()`` raises immediately so that a mis-built GPU box fails loudly
instead of silently computing something else.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime libamdhip64.so.7 before our library)

from . import knobs

_HERE = os.path.dirname(os.path.abspath(__file__))
# KRRN_HIP_LIB: an alternative build of the same library (kernel-variant experiments)
LIB_PATH = knobs.text("KRRN_HIP_LIB") or os.path.join(_HERE, "libkrrn_hip.so")

_lock = threading.Lock()
_lib = None

_ERRORS = {-1: "KRRN_EARG (null pointer / bad argument)",
           -2: "KRRN_ESHAPE (dimension outside the supported range)",
           -3: "KRRN_EALIGN (16-byte alignment / channel stride violation)",
           -4: "KRRN_EUNSUPPORTED (hipBLASLt rejected the problem)"}

# name -> (argtypes). Every entry point returns int.
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_U64 = ctypes.c_uint64
SIGNATURES = {
    "krrn_conv2d_f32": [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I, _P, _P, _P, _I,
                        _P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P],
}


def register(name, argtypes):
    SIGNATURES[name] = argtypes


def lib():
    """Return the loaded library (raises RuntimeError when it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(the KRRN HIP path has no fallback)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, argtypes in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.argtypes = argtypes
                fn.restype = ctypes.c_int
            _lib = handle
    return _lib


def check(status: int, name: str):
    if status != 0:
        msg = _ERRORS.get(status, f"hipError_t {status}")
        raise RuntimeError(f"{name} failed: {msg}")


def call(name: str, *args):
    fn = getattr(lib(), name)
    check(fn(*args), name)
