"""Back-propagatable PnP on the GPU, the drop-in for
lib/network/dnn/BPnP.py: `BPnP` (torch.autograd.Function) and `BPnPModle` (nn.Module) with the
reference's arguments and result.

    P_6d = BPnP.apply(pts2d [bs, n, 2], pts3d [n, 3], K [3, 3], ini_pose=None)  # [bs, 6]

P_6d = (angle-axis, t) per crop. Forward (BPnP.py:24-51): without `ini_pose` the initial pose
is PnP-RANSAC with a 3 px threshold (the reference's cv2.solvePnPRansac, here the batched
EPnP-RANSAC kernel, krrn_pnp_ransac_f32), then Levenberg-Marquardt on all points
(cv2.solvePnP ITERATIVE with the guess: krrn_bpnp_solve_f32). Backward (BPnP.py:53-117): the
implicit-function gradients w.r.t. pts2d, pts3d and K (krrn_bpnp_backward_f32); grad_z and grad_K
are summed over the batch like the reference. pts3d may also be [bs, n, 3] (one set per crop).
All tensors on the GPU; there is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib
from .runtime import P, ptr

_I = ctypes.c_int
_lib.register("krrn_bpnp_solve_f32", [P, P, _I, P, P, P, _I, _I, _I, P, P, P])
_lib.register("krrn_bpnp_backward_f32", [P, P, P, _I, P, P, _I, _I, P, P, P, P, P])

LM_ITERS = 50
RANSAC_THR = 3.0  # reprojectionError of the reference's solvePnPRansac (BPnP.py:36-38)
PNP_MAX_P = 1024  # kPnpMaxP of krrn_pnp_ransac_f32 (csrc/pnp.hip): larger sets are subsampled


def _stream(dev):
    return P(torch.cuda.current_stream(dev).cuda_stream)


def _check_inputs(pts2d, pts3d, K):
    if not (pts2d.is_cuda and pts3d.is_cuda and K.is_cuda):
        raise RuntimeError("BPnP runs on the HIP path only (GPU tensors expected)")
    bs, n = pts2d.shape[0], pts2d.shape[1]
    if pts2d.shape != (bs, n, 2) or K.shape != (3, 3):
        raise ValueError(f"pts2d [bs, n, 2] and K [3, 3] expected, got {tuple(pts2d.shape)}, {tuple(K.shape)}")
    if pts3d.shape not in ((n, 3), (bs, n, 3)):
        raise ValueError(f"pts3d [n, 3] or [bs, n, 3] expected, got {tuple(pts3d.shape)}")
    return bs, n, int(pts3d.dim() == 3)


def ransac_init(pts2d: torch.Tensor, pts3d: torch.Tensor, K: torch.Tensor):
    """Initial R [bs, 3, 3], t [bs, 3] from the batched EPnP-RANSAC kernel (thr 3 px)."""
    from .pose import get_pose
    bs, n, per_crop = _check_inputs(pts2d, pts3d, K)
    dev = pts2d.device
    z = pts3d if per_crop else pts3d.expand(bs, n, 3)
    xyz = z.permute(0, 2, 1).contiguous().view(bs, 3, 1, n)  # model coords as a 1 x n "map"
    Kf = K.detach().double().cpu()
    data = {"choose": torch.arange(n, device=dev).view(1, 1, n).expand(bs, 1, n).contiguous(),
            "x_map_choosed": pts2d[:, :, 0].contiguous(), "y_map_choosed": pts2d[:, :, 1].contiguous(),
            "intrinsic": torch.tensor([[Kf[0, 0], Kf[1, 1], Kf[0, 2], Kf[1, 2]]], dtype=torch.float32,
                                      device=dev).expand(bs, 4).contiguous(),
            "extent": torch.ones(bs, 3, dtype=torch.float64, device=dev),
            "lfborder": torch.zeros(bs, 3, dtype=torch.float64, device=dev)}
    P_ = min(n, PNP_MAX_P)
    sel = torch.stack([torch.randperm(n)[:P_] for _ in range(bs)]).to(torch.int32)
    return get_pose({"xyz": xyz}, data, num_points=P_, thr=RANSAC_THR, sel=sel)


def solve(pts2d: torch.Tensor, pts3d: torch.Tensor, K: torch.Tensor, ini_pose: torch.Tensor = None,
          iters: int = LM_ITERS, return_cost: bool = False):
    """BPnP.forward: P_6d [bs, 6]."""
    bs, n, per_crop = _check_inputs(pts2d, pts3d, K)
    dev = pts2d.device
    x = pts2d.detach().float().contiguous()
    z = pts3d.detach().float().contiguous()
    Kc = K.detach().float().contiguous()
    R0 = None
    if ini_pose is None:
        R0, t0 = ransac_init(x, z, Kc)
        y0 = torch.cat([torch.zeros(bs, 3, device=dev), t0.float()], dim=1).contiguous()
        R0 = R0.float().contiguous()
    else:
        y0 = ini_pose.detach().float().reshape(bs, 6).contiguous()
    y = torch.empty(bs, 6, dtype=torch.float32, device=dev)
    cost = torch.empty(bs, dtype=torch.float32, device=dev)
    _lib.call("krrn_bpnp_solve_f32", ptr(x), ptr(z), per_crop, ptr(Kc), ptr(y0), ptr(R0), bs, n, iters, ptr(y),
              ptr(cost), _stream(dev))
    return (y, cost) if return_cost else y


def backward(pts2d, P_6d, pts3d, K, grad_output):
    """BPnP.backward: (grad_x [bs, n, 2], grad_z like pts3d, grad_K [3, 3])."""
    bs, n, per_crop = _check_inputs(pts2d, pts3d, K)
    dev = pts2d.device
    x = pts2d.detach().float().contiguous()
    y = P_6d.detach().float().contiguous()
    z = pts3d.detach().float().contiguous()
    Kc = K.detach().float().contiguous()
    g = grad_output.detach().float().contiguous()
    gx = torch.empty(bs, n, 2, dtype=torch.float32, device=dev)
    gz = torch.empty(z.shape, dtype=torch.float32, device=dev)
    gK = torch.empty(3, 3, dtype=torch.float32, device=dev)
    ws = torch.empty(bs * (3 * n + 9), dtype=torch.float64, device=dev)
    _lib.call("krrn_bpnp_backward_f32", ptr(x), ptr(y), ptr(z), per_crop, ptr(Kc), ptr(g), bs, n, ptr(gx), ptr(gz),
              ptr(gK), ptr(ws), _stream(dev))
    return gx.to(pts2d.dtype), gz.to(pts3d.dtype), gK.to(K.dtype)


class BPnP(torch.autograd.Function):
    """Drop-in for lib/network/dnn/BPnP.py:8-117 (forward / backward as above)."""

    @staticmethod
    def forward(ctx, pts2d, pts3d, K, ini_pose=None):
        P_6d = solve(pts2d, pts3d, K, ini_pose)
        ctx.save_for_backward(pts2d, P_6d, pts3d, K)
        return P_6d

    @staticmethod
    def backward(ctx, grad_output):
        pts2d, P_6d, pts3d, K = ctx.saved_tensors
        gx, gz, gK = backward(pts2d, P_6d, pts3d, K, grad_output)
        return gx, gz, gK, None


class BPnPModle(nn.Module):
    """lib/network/dnn/BPnP.py:120-125 (the reference's class name, kept for drop-in use)."""

    def forward(self, pts2d, pts3d, K, ini_pose=None):
        return BPnP.apply(pts2d, pts3d, K, ini_pose)
