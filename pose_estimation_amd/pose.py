"""Rotation by PnP-RANSAC on the reconstructed correspondences: Trainer.get_pose
(tools/trainer.py:383-438), batched and on the GPU (krrn_pnp_ransac_f32).

    R, t = get_pose(pred, data)          # R [B, 3, 3], t [B, 3] (PnP translation)

Reference semantics kept: 256 of the N chosen pixels per crop (torch.randperm on the CPU
generator, :406-408), object points = xyz * extent + lfborder (f64, :415-421), image points
= full-frame (x, y) of the same pixels, EPnP hypotheses, 1 px reprojection threshold,
EPnP refinement on the inliers, R as a matrix (the rvec -> kornia Rodrigues step is an
identity on R). The reference asserts B == 1 (:402); any B works here, one workgroup per crop.
RANSAC: H = 100 hypotheses per crop (cv2's default iterationsCount), drawn on the device
(krrn_ransac_subsets) unless given explicitly, scored in parallel and selected by cv2's own loop
(in order, stopping at its adaptive iteration count for confidence 0.9999, :426).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .runtime import P, Plan, h2d, ptr
from . import _lib

NUM_POINTS = 256
N_HYP = 100
THRESHOLD = 1.0
CONFIDENCE = 0.9999

_seeds: Dict[int, torch.Tensor] = {}


def _seed(device) -> torch.Tensor:
    idx = device.index or 0
    if idx not in _seeds:
        _seeds[idx] = torch.zeros(1, dtype=torch.int64, device=device)
    return _seeds[idx]


def _dev(t: torch.Tensor, device, dtype=None) -> torch.Tensor:
    return h2d(t, device, dtype)


def draw_sel(B: int, N: int, num_points: int = NUM_POINTS) -> torch.Tensor:
    """torch.randperm(N)[:num_points] per crop on the CPU generator (trainer.py:406-408)."""
    return torch.stack([torch.randperm(N)[:num_points] for _ in range(B)]).to(torch.int32)


def get_pose(pred, data, num_points: int = NUM_POINTS, n_hyp: int = N_HYP, thr: float = THRESHOLD,
             sel: Optional[torch.Tensor] = None, subsets: Optional[torch.Tensor] = None, return_info: bool = False):
    xyz = pred["xyz"]
    if not xyz.is_cuda:
        raise RuntimeError("get_pose runs on the HIP path only (pred['xyz'] must be a GPU tensor)")
    dev = xyz.device
    xyz = xyz.contiguous()
    B, _, H, W = xyz.shape
    choose = _dev(data["choose"].reshape(B, -1), dev, torch.int64)
    N = choose.shape[1]
    P_ = min(num_points, N)
    if sel is None:
        sel = draw_sel(B, N, P_)
    sel = _dev(sel.reshape(B, P_), dev, torch.int32)
    xm = _dev(data["x_map_choosed"].reshape(B, N), dev, torch.float32)
    ym = _dev(data["y_map_choosed"].reshape(B, N), dev, torch.float32)
    K4 = _dev(data["intrinsic"].reshape(B, 4), dev, torch.float32)
    ext = _dev(data["extent"].reshape(B, 3), dev, torch.float64)
    lfb = _dev(data["lfborder"].reshape(B, 3), dev, torch.float64)
    stream = P(torch.cuda.current_stream(dev).cuda_stream)
    lib = _lib.lib()
    if subsets is None:
        subsets = torch.empty((B, n_hyp, 5), dtype=torch.int32, device=dev)
        seed = _seed(dev)
        _lib.check(lib.krrn_ransac_subsets(ptr(seed), 7, B, n_hyp, P_, ptr(subsets), stream), "krrn_ransac_subsets")
        _lib.check(lib.krrn_rng_advance(ptr(seed), stream), "krrn_rng_advance")
    else:
        subsets = _dev(subsets.reshape(B, -1, 5), dev, torch.int32)
        n_hyp = subsets.shape[1]
    R = torch.empty((B, 3, 3), dtype=torch.float32, device=dev)
    t = torch.empty((B, 3), dtype=torch.float32, device=dev)
    inl = torch.empty((B,), dtype=torch.int32, device=dev)
    mask = torch.empty((B, P_), dtype=torch.uint8, device=dev)
    ws = torch.empty((B * n_hyp * 13,), dtype=torch.float32, device=dev)
    _lib.check(lib.krrn_pnp_ransac_f32(ptr(xyz), H * W, ptr(choose), N, ptr(sel), P_, ptr(xm), ptr(ym), ptr(K4),
                                       ptr(ext), ptr(lfb), ptr(subsets), n_hyp, float(thr), CONFIDENCE, ptr(ws), ptr(R), ptr(t),
                                       ptr(inl), ptr(mask), B, stream), "krrn_pnp_ransac_f32")
    if return_info:
        return R, t, {"inliers": inl, "mask": mask, "sel": sel, "subsets": subsets, "workspace": ws}
    return R, t


def add_pose_ops(plan: Plan, xyz: torch.Tensor, choose: torch.Tensor, B: int, N: int, xm: torch.Tensor,
                 ym: torch.Tensor, K4: torch.Tensor, ext: torch.Tensor, lfb: torch.Tensor, seed: torch.Tensor,
                 num_points: int = NUM_POINTS, n_hyp: int = N_HYP, thr: float = THRESHOLD):
    """Append the pose step to a plan (graph-capturable: choose subset and RANSAC subsets drawn
    on the device). Returns (R, t, inliers) buffers."""
    H, W = xyz.shape[2], xyz.shape[3]
    P_ = min(num_points, N)
    sel = plan.buf((B, P_), torch.int32)
    subsets = plan.buf((B, n_hyp, 5), torch.int32)
    R = plan.buf((B, 3, 3))
    t = plan.buf((B, 3))
    inl = plan.buf((B,), torch.int32)
    mask = plan.buf((B, P_), torch.uint8)
    ws = plan.buf((B * n_hyp * 13,))
    plan.add("krrn_randperm_i32", ptr(seed), 5, N, P_, B, ptr(sel))
    plan.add("krrn_ransac_subsets", ptr(seed), 6, B, n_hyp, P_, ptr(subsets))
    plan.add("krrn_pnp_ransac_f32", ptr(xyz), H * W, ptr(choose), N, ptr(sel), P_, ptr(xm), ptr(ym), ptr(K4), ptr(ext),
             ptr(lfb), ptr(subsets), n_hyp, float(thr), CONFIDENCE, ptr(ws), ptr(R), ptr(t), ptr(inl), ptr(mask), B)
    return R, t, inl, dict(sel=sel, subsets=subsets, mask=mask)
