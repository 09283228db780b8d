"""Farthest point sampling on the GPU: tools/script/sample_model.py:35-48,
the offline sampler of the FPS region centres (kps_orb9_fps / the 64 region points of the region
head, batchdataset.py:723-728). One workgroup per point set (krrn_fps_f32).

    idx = farthest_point_sampling(points, n_samples)   # points [n, 3] or [B, n, 3] on the GPU
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .runtime import P, ptr

_lib.register("krrn_fps_f32", [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P])


def farthest_point_sampling(points: torch.Tensor, n_samples: int) -> torch.Tensor:
    if not points.is_cuda:
        raise RuntimeError("farthest_point_sampling runs on the HIP path only (GPU tensor expected)")
    single = points.dim() == 2
    pts = (points[None] if single else points).to(torch.float32).contiguous()
    B, n, _ = pts.shape
    out = torch.empty((B, n_samples), dtype=torch.int32, device=pts.device)
    _lib.call("krrn_fps_f32", ptr(pts), B, n, n_samples, ptr(out), P(torch.cuda.current_stream(pts.device).cuda_stream))
    out = out.long()
    return out[0] if single else out
