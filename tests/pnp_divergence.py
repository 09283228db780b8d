"""Dissects where the kernel-order EPnP-RANSAC (oracle_pnp_ransac, count-for-count equal to the GPU
kernel: tests/test_gpu_pnp.py::test_full_ransac_matches_oracle) and the OpenCV-semantics restatement
(oracle_pnp_ransac_cv: cyclic Jacobi, SVD beta solves, QR Gauss-Newton, det fix by negating R's
third row) part ways on noisy scenes. Test infrastructure (CPU only, uses oracle/).

For every crop it scores all H hypotheses under both numerics (oracle_pnp_hypotheses_diag), runs
ptsetreg.cpp's selection loop on each count list, and classifies a difference in the selected count:

  same-h      both loops select the same hypothesis; its inlier count differs (threshold points
              flipping under two slightly different 5-point poses)
  flip        a hypothesis' count differs a lot between the numerics (a different beta approximation
              won, or only one side's Procrustes corrected a reflection) and that decides the selection
  niters      every hypothesis up to both loops' stop scores within a few points, but one count change
              lowers cv2's adaptive iteration count (RANSACUpdateNumIters) so one loop stops before the
              other's winner

python tests/pnp_divergence.py [n_seeds] prints the per-hypothesis statistics and every divergent crop.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pnp as opnp  # noqa: E402

K4 = np.array([572.4114, 573.57043, 325.2611, 242.04899], np.float32)
EXT = np.array([0.067, 0.1276, 0.1175])
LFB = np.array([-0.0335, -0.0638, -0.0587])


def scene_points(rng, P=256, noise_px=0.4, outlier_frac=0.3):
    """One crop's 256 RANSAC correspondences the way tests/test_gpu_pnp.py::_scene builds them
    (f32 normalised model coordinates -> metres, projected under a random pose, noise, outliers)."""
    R = opnp.rotation_from_axis_angle(rng.normal(size=3))
    t = np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.7, 1.1)])
    u32 = rng.random((P, 3)).astype(np.float32)
    pw = u32.astype(np.float64) * EXT + LFB
    pc = pw @ R.T + t
    img = np.stack([K4[0] * pc[:, 0] / pc[:, 2] + K4[2], K4[1] * pc[:, 1] / pc[:, 2] + K4[3]], 1)
    img += rng.normal(scale=noise_px, size=img.shape) if noise_px else 0
    out = rng.random(P) < outlier_frac
    img[out] += rng.uniform(-20, 20, size=(out.sum(), 2))
    obj = (u32.astype(np.float64) * EXT + LFB).astype(np.float32)
    return obj, img.astype(np.float32), R, t


def hypotheses(obj, img, subsets, cv, thr=1.0):
    """(R [H,3,3], t [H,3], counts [H], approx [H], detneg [H], any_detneg [H]) under one numerics."""
    lib = opnp._load()
    f = lib.oracle_pnp_hypotheses_diag
    f.restype = None
    H = len(subsets)
    R = np.zeros((H, 9), np.float32)
    t = np.zeros((H, 3), np.float32)
    cnt = np.zeros(H, np.int32)
    diag = np.zeros(H, np.int32)
    sub = np.ascontiguousarray(subsets, np.int32)
    f(opnp._p(np.ascontiguousarray(obj)), opnp._p(np.ascontiguousarray(img)), ctypes.c_int(len(obj)),
      opnp._p(K4), opnp._p(sub), ctypes.c_int(H), ctypes.c_float(thr), ctypes.c_int(int(cv)),
      opnp._p(R), opnp._p(t), opnp._p(cnt), opnp._p(diag))
    return R.reshape(H, 3, 3), t, cnt, diag & 3, (diag >> 2) & 1, (diag >> 3) & 1


def update_niters(conf, ep, model_points, max_iters):
    """cv::RANSACUpdateNumIters (ptsetreg.cpp)."""
    conf, ep = min(max(conf, 0.0), 1.0), min(max(ep, 0.0), 1.0)
    num = max(1.0 - conf, np.finfo(np.float64).tiny)
    denom = 1.0 - (1.0 - ep) ** model_points
    if denom < np.finfo(np.float64).tiny:
        return 0
    num, denom = np.log(num), np.log(denom)
    return max_iters if (denom >= 0 or -num >= max_iters * (-denom)) else int(np.rint(num / denom))


def select(cnts, P, conf=0.9999):
    """ptsetreg.cpp's loop over scored hypotheses -> (best h, best count, hypotheses visited)."""
    best, best_cnt, niters, h = -1, 0, len(cnts), 0
    while h < niters:
        c = int(cnts[h])
        if c > max(best_cnt, 4):
            best, best_cnt = h, c
            niters = update_niters(conf, (P - c) / P, 5, niters)
        h += 1
    return best, best_cnt, h


def classify(ck, cc, P, small=3):
    """Why the two selections differ (None when they select the same count)."""
    bk, nk, ik = select(ck, P)
    bc, nc, ic = select(cc, P)
    if nk == nc:
        return None
    if bk == bc:
        return "same-h"
    d = np.abs(ck.astype(int) - cc)
    if d[[bk, bc]].max() > small:
        return "flip"
    # both winners score alike under both numerics: one loop stopped before the other's winner
    return "niters" if min(ik, ic) <= max(bk, bc) else "flip"


def dissect(n_seeds=40, B=16, H=100, noise_px=0.4, outlier_frac=0.3, verbose=True):
    stats = {"hyps": 0, "hyp_diff": 0, "hyp_diff_gt3": 0, "approx_diff": 0, "det_diff": 0,
             "big_with_approx_or_det": 0, "crops": 0, "sel_diff": 0, "same-h": 0, "flip": 0, "niters": 0,
             "max_sel_gap": 0, "gpu_minus_cv": []}
    for seed in range(n_seeds):
        rng = np.random.default_rng(10_000 + seed)
        for b in range(B):
            obj, img, _, _ = scene_points(rng, noise_px=noise_px, outlier_frac=outlier_frac)
            subs = np.stack([rng.permutation(len(obj))[:5] for _ in range(H)]).astype(np.int32)
            _, _, ck, ak, dk, _ = hypotheses(obj, img, subs, cv=False)
            _, _, cc, ac, dc, _ = hypotheses(obj, img, subs, cv=True)
            diff = ck != cc
            big = np.abs(ck.astype(int) - cc) > 3
            stats["hyps"] += H
            stats["hyp_diff"] += int(diff.sum())
            stats["hyp_diff_gt3"] += int(big.sum())
            stats["approx_diff"] += int((ak != ac).sum())
            stats["det_diff"] += int((dk != dc).sum())
            stats["big_with_approx_or_det"] += int((big & ((ak != ac) | (dk != dc))).sum())
            stats["crops"] += 1
            why = classify(ck, cc, len(obj))
            _, nk, _ = select(ck, len(obj))
            _, nc, _ = select(cc, len(obj))
            stats["gpu_minus_cv"].append(nk - nc)
            if why is not None:
                stats["sel_diff"] += 1
                stats[why] += 1
                stats["max_sel_gap"] = max(stats["max_sel_gap"], abs(nk - nc))
                if verbose:
                    bk, _, ik = select(ck, len(obj))
                    bc, _, ic = select(cc, len(obj))
                    print(f"seed {seed} crop {b}: kernel-order h={bk} n={nk} (visited {ik}), "
                          f"cv h={bc} n={nc} (visited {ic}) -> {why}; at those h: kernel {ck[[bk, bc]]}, "
                          f"cv {cc[[bk, bc]]}, approx k/cv {ak[[bk, bc]]}/{ac[[bk, bc]]}, "
                          f"detneg k/cv {dk[[bk, bc]]}/{dc[[bk, bc]]}")
    g = np.array(stats.pop("gpu_minus_cv"))
    stats["sel_gap_mean"] = float(g.mean())
    stats["sel_gap_hist"] = {int(k): int(v) for k, v in zip(*np.unique(g, return_counts=True))}
    return stats


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    s = dissect(n)
    for k, v in s.items():
        print(f"{k}: {v}")


def ingredient_sweep(n_seeds=20, B=16, H=100, noise_px=0.4, outlier_frac=0.3):
    """Agreement of the OpenCV-semantics EPnP with the kernel-order one as single ingredients are
    swapped for the kernel's (oracle_set_cv_variant bits: 1 = null-space basis from the kernel's
    Jacobi, 2 = Kabsch, 4 = Cholesky solves) -> {variant: (hypotheses with equal counts, with a
    count gap > 3, crops whose selected count differs)}."""
    lib = opnp._load()
    out = {}
    try:
        for v in range(8):
            lib.oracle_set_cv_variant(ctypes.c_int(v))
            eq = big = sel = tot = 0
            for seed in range(n_seeds):
                rng = np.random.default_rng(10_000 + seed)
                for b in range(B):
                    obj, img, _, _ = scene_points(rng, noise_px=noise_px, outlier_frac=outlier_frac)
                    subs = np.stack([rng.permutation(len(obj))[:5] for _ in range(H)]).astype(np.int32)
                    ck = hypotheses(obj, img, subs, cv=False)[2]
                    cc = hypotheses(obj, img, subs, cv=True)[2]
                    eq += int((ck == cc).sum())
                    big += int((np.abs(ck.astype(int) - cc) > 3).sum())
                    sel += int(select(ck, len(obj))[1] != select(cc, len(obj))[1])
                    tot += H
            out[v] = (eq / tot, big / tot, sel / (n_seeds * B))
    finally:
        lib.oracle_set_cv_variant(ctypes.c_int(0))
    return out
