"""ORACLE (test infrastructure only): ctypes binding of oracle/pnp_ref.c.

Restates cv2.solvePnPRansac(EPNP, confidence=0.9999, reprojectionError=1) as called at
tools/trainer.py:423-427 (see the header of pnp_ref.c for what is and is not pinned).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libpnp_oracle.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _lib = ctypes.CDLL(_SO)
        _lib.oracle_epnp.restype = ctypes.c_double
        _lib.oracle_epnp.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] + [ctypes.c_void_p] * 3
        _lib.oracle_pnp_ransac.restype = ctypes.c_int
        _lib.oracle_pnp_ransac.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def epnp(pw, uv, K4):
    """EPnP on all correspondences (float64). Returns (R[3,3], t[3], mean reprojection error)."""
    pw = np.ascontiguousarray(pw, dtype=np.float64)
    uv = np.ascontiguousarray(uv, dtype=np.float64)
    K4 = np.ascontiguousarray(K4, dtype=np.float64)
    R = np.zeros(9)
    t = np.zeros(3)
    err = _load().oracle_epnp(_p(pw), _p(uv), len(pw), _p(K4), _p(R), _p(t))
    return R.reshape(3, 3), t, err


def pnp_ransac(obj, img, K4, subsets, thr=1.0, conf=0.9999):
    """One crop: obj [P,3] f32, img [P,2] f32, K4 (fx, fy, cx, cy), subsets [H,5] int (H =
    iterationsCount; the loop stops early at cv2's adaptive count for `conf`).

    Returns (R [3,3] f32, t [3] f32, inlier_count, inlier_mask [P] bool, best_h)."""
    obj = np.ascontiguousarray(obj, dtype=np.float32)
    img = np.ascontiguousarray(img, dtype=np.float32)
    K4 = np.ascontiguousarray(K4, dtype=np.float32)
    subsets = np.ascontiguousarray(subsets, dtype=np.int32)
    R = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    mask = np.zeros(len(obj), np.uint8)
    best = ctypes.c_int(-1)
    cnt = _load().oracle_pnp_ransac(_p(obj), _p(img), len(obj), _p(K4), _p(subsets), len(subsets), float(thr),
                                    float(conf), _p(R), _p(t), _p(mask), ctypes.byref(best))
    return R.reshape(3, 3), t, cnt, mask.astype(bool), best.value


def pnp_ransac_cv(obj, img, K4, subsets, thr=1.0, conf=0.9999):
    """pnp_ransac with the OpenCV-semantics EPnP of pnp_ref.c (cyclic 12 x 12 Jacobi, SVD beta
    solves, QR Gauss-Newton, U V^T with the det fix): numerics independent of the kernel's.
    Returns (R [3,3] f32, t [3] f32, inlier_count, best_h)."""
    obj = np.ascontiguousarray(obj, dtype=np.float32)
    img = np.ascontiguousarray(img, dtype=np.float32)
    K4 = np.ascontiguousarray(K4, dtype=np.float32)
    subsets = np.ascontiguousarray(subsets, dtype=np.int32)
    R = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    best = ctypes.c_int(-1)
    lib = _load()
    lib.oracle_pnp_ransac_cv.restype = ctypes.c_int
    lib.oracle_pnp_ransac_cv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    cnt = lib.oracle_pnp_ransac_cv(_p(obj), _p(img), len(obj), _p(K4), _p(subsets), len(subsets), float(thr),
                                   float(conf), _p(R), _p(t), ctypes.byref(best))
    return R.reshape(3, 3), t, cnt, best.value


def pnp_hypotheses(obj, img, K4, subsets, thr=1.0):
    """Diagnostics: every RANSAC hypothesis -> (R [H,3,3] f32, t [H,3] f32, counts [H])."""
    obj = np.ascontiguousarray(obj, dtype=np.float32)
    img = np.ascontiguousarray(img, dtype=np.float32)
    K4 = np.ascontiguousarray(K4, dtype=np.float32)
    subsets = np.ascontiguousarray(subsets, dtype=np.int32)
    H = len(subsets)
    R = np.zeros((H, 9), np.float32)
    t = np.zeros((H, 3), np.float32)
    cnt = np.zeros(H, np.int32)
    lib = _load()
    lib.oracle_pnp_hypotheses.restype = None
    lib.oracle_pnp_hypotheses(_p(obj), _p(img), ctypes.c_int(len(obj)), _p(K4), _p(subsets), ctypes.c_int(H),
                              ctypes.c_float(thr), _p(R), _p(t), _p(cnt))
    return R.reshape(H, 3, 3), t, cnt


def rotation_from_axis_angle(rvec):
    """Rodrigues (kornia.angle_axis_to_rotation_matrix semantics, float64)."""
    rvec = np.asarray(rvec, dtype=np.float64)
    th = np.linalg.norm(rvec)
    if th < 1e-12:
        return np.eye(3)
    k = rvec / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
