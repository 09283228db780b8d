"""Pose-accuracy harness: Metric (lib/utils/metric.py:13-113) and Trainer.cal_dis
(tools/trainer.py:370-381) — the ADD(-S) / AUC half of BASELINE.json's metric.

ADD / ADD-S (the reference broadcasts an [N, N, 3] tensor for ADD-S, metric.py:27-31) run for a
whole batch of crops in one HIP launch (krrn_add_metric_f32: model points transformed on the
fly, exact direct-difference norms, min over predictions per target); quaternion angle,
translation error and AUC are vectorised host bookkeeping.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

import ctypes

from . import _lib
from .runtime import P, h2d, ptr

_I = ctypes.c_int
_lib.register("krrn_add_metric_f32", [P, P, P, P, P, P, _I, _I, _I, P, P, P])


def add_metric(pred_r: torch.Tensor, pred_t: torch.Tensor, model_points: torch.Tensor, target: torch.Tensor,
               cls_id: torch.Tensor, sym: Sequence[int]) -> torch.Tensor:
    """f64 [B]: ADD, or ADD-S for crops whose cls_id is in `sym`, of pred = mp @ R^T + t against
    target (metric.py:17-35 per crop), one krrn_add_metric_f32 launch for the batch."""
    dev = pred_t.device
    if dev.type != "cuda":
        raise RuntimeError("add_metric runs on the HIP path only (GPU tensors)")
    B, Pn = model_points.shape[0], model_points.shape[1]
    f = lambda x: h2d(x, dev, torch.float32)  # noqa: E731
    # every converted operand stays bound until the launch is enqueued: a temporary freed after
    # ptr() could hand its caching-allocator block to the next conversion before the kernel reads it
    r, t, mp, tg = f(pred_r).reshape(B, 9), f(pred_t).reshape(B, 3), f(model_points), f(target)
    cls = h2d(cls_id.reshape(B), dev, torch.int64)
    symt = h2d(torch.tensor(list(sym) or [0], dtype=torch.int32), dev)
    ws = torch.empty((B * ((Pn + 255) // 256),), dtype=torch.float64, device=dev)
    out = torch.empty((B,), dtype=torch.float64, device=dev)
    _lib.call("krrn_add_metric_f32", ptr(r), ptr(t), ptr(mp), ptr(tg), ptr(cls), ptr(symt),
              len(sym), B, Pn, ptr(ws), ptr(out), P(torch.cuda.current_stream(dev).cuda_stream))
    return out


def rotation_matrix_to_quaternion(R: torch.Tensor) -> torch.Tensor:
    """(w, x, y, z) from a rotation matrix (Shepperd's method, the kornia conversion used at
    metric.py:70-72)."""
    R = R.double()
    m00, m01, m02 = R[..., 0, 0], R[..., 0, 1], R[..., 0, 2]
    m10, m11, m12 = R[..., 1, 0], R[..., 1, 1], R[..., 1, 2]
    m20, m21, m22 = R[..., 2, 0], R[..., 2, 1], R[..., 2, 2]
    tr = m00 + m11 + m22
    eps = 1e-12
    s0 = torch.sqrt((tr + 1.0).clamp_min(eps)) * 2
    q0 = torch.stack([0.25 * s0, (m21 - m12) / s0, (m02 - m20) / s0, (m10 - m01) / s0], -1)
    s1 = torch.sqrt((1.0 + m00 - m11 - m22).clamp_min(eps)) * 2
    q1 = torch.stack([(m21 - m12) / s1, 0.25 * s1, (m01 + m10) / s1, (m02 + m20) / s1], -1)
    s2 = torch.sqrt((1.0 + m11 - m00 - m22).clamp_min(eps)) * 2
    q2 = torch.stack([(m02 - m20) / s2, (m01 + m10) / s2, 0.25 * s2, (m12 + m21) / s2], -1)
    s3 = torch.sqrt((1.0 + m22 - m00 - m11).clamp_min(eps)) * 2
    q3 = torch.stack([(m10 - m01) / s3, (m02 + m20) / s3, (m12 + m21) / s3, 0.25 * s3], -1)
    c0 = (tr > 0)[..., None]
    c1 = ((m00 > m11) & (m00 > m22))[..., None]
    c2 = (m11 > m22)[..., None]
    return torch.where(c0, q0, torch.where(c1, q1, torch.where(c2, q2, q3)))


class Metric:
    def __init__(self, sym: Sequence[int]):
        self.sys = list(sym)

    def cal_adds_cuda(self, pred: torch.Tensor, target: torch.Tensor, idx: int) -> Tuple[float, float]:
        """metric.py:17-35 for one crop's already-transformed points (identity pose through the
        batched kernel)."""
        assert pred.dim() == target.dim() == 2
        dev = pred.device
        eye = torch.eye(3, device=dev).view(1, 3, 3)
        zero = torch.zeros((1, 3), device=dev)
        v = float(add_metric(eye, zero, pred.unsqueeze(0), target.unsqueeze(0),
                             torch.tensor([int(idx)], device=dev), self.sys)[0])
        return v, v

    def cal_auc(self, add_dis: List[float], max_dis: float = 0.1) -> float:
        D = np.array(add_dis, dtype=np.float64)
        D[np.where(D > max_dis)] = np.inf
        D = np.sort(D)
        n = len(add_dis)
        acc = np.cumsum(np.ones((1, n)), dtype=np.float32) / n
        return self.voc_ap(D, acc) * 100.0

    @staticmethod
    def voc_ap(rec, prec):
        idx = np.where(rec != np.inf)
        if len(idx[0]) == 0:
            return 0
        rec = rec[idx]
        prec = prec[idx]
        mrec = np.array([0.0] + list(rec) + [0.1])
        mpre = np.array([0.0] + list(prec) + [prec[-1]])
        n = prec.shape[0]  # the running max over mpre[1 .. n-1] (metric.py:61-62), as one scan
        mpre[:n] = np.maximum.accumulate(mpre[:n])
        i = np.where(mrec[1:] != mrec[0:-1])[0] + 1
        return np.sum((mrec[i] - mrec[i - 1]) * mpre[i]) * 10

    @staticmethod
    def angular_distance(R1: torch.Tensor, R2: torch.Tensor, eps: float = 1e-7) -> torch.Tensor:
        q1 = torch.nn.functional.normalize(rotation_matrix_to_quaternion(R1), p=2.0, dim=-1, eps=1e-12)
        q2 = torch.nn.functional.normalize(rotation_matrix_to_quaternion(R2), p=2.0, dim=-1, eps=1e-12)
        dot = q1.reshape(-1, 4) @ q2.reshape(-1, 4).t()
        return 2 * torch.acos(torch.clamp(dot.abs(), -1.0 + eps, 1.0 - eps)) / torch.pi * 180.0

    @staticmethod
    def translation_distance(t1, t2):
        return torch.norm(t1 - t2, dim=-1)


def rt_errors(pred_r: torch.Tensor, pred_t: torch.Tensor, target_r: torch.Tensor, target_t: torch.Tensor):
    """(rotation error deg [B], translation error m [B]) as f64 numpy arrays (trainer.py:376-380:
    metric.angular_distance / translation_distance on the CPU)."""
    B = pred_t.shape[0]
    R = pred_r.detach().float().cpu().reshape(B, 3, 3)
    Rt = target_r.detach().float().cpu().reshape(B, 3, 3)
    q1 = torch.nn.functional.normalize(rotation_matrix_to_quaternion(R), p=2.0, dim=-1, eps=1e-12)
    q2 = torch.nn.functional.normalize(rotation_matrix_to_quaternion(Rt), p=2.0, dim=-1, eps=1e-12)
    dot = (q1 * q2).sum(-1)
    eps = 1e-7
    r = (2 * torch.acos(torch.clamp(dot.abs(), -1.0 + eps, 1.0 - eps)) / torch.pi * 180.0).numpy()
    t = torch.norm(pred_t.detach().float().cpu().reshape(B, 3) - target_t.detach().float().cpu().reshape(B, 3),
                   dim=-1).double().numpy()
    return r, t


def cal_dis_batch(metric: Metric, pred_r: torch.Tensor, pred_t: torch.Tensor, datas):
    """Trainer.cal_dis (trainer.py:370-381) for every crop of a batch: (ADD(-S) [B], rotation error
    deg [B], translation error m [B]) as f64 numpy arrays."""
    B = pred_t.shape[0]
    add = add_metric(pred_r, pred_t.reshape(B, 3), datas["model_points"], datas["target"], datas["cls_id"],
                     metric.sys).cpu().numpy()
    r, t = rt_errors(pred_r, pred_t, datas["target_r"], datas["target_t"])
    return add, r, t


def cal_dis(metric: Metric, pred_r: torch.Tensor, pred_t: torch.Tensor, datas, b: int = 0):
    """Trainer.cal_dis for crop b: (ADD or ADD-S, rotation error deg, translation error m)."""
    dev = pred_t.device
    mp = datas["model_points"][b].to(dev)
    target = datas["target"][b].to(dev)
    R = pred_r[b].to(dev).float()
    pts = mp @ R.t() + pred_t[b].reshape(1, 3).to(dev)
    add, _ = metric.cal_adds_cuda(pts, target, int(datas["cls_id"][b]))
    r = float(metric.angular_distance(R.cpu().reshape(1, 3, 3), datas["target_r"][b].cpu().reshape(1, 3, 3)).squeeze())
    t = float(metric.translation_distance(pred_t[b].cpu().reshape(3), datas["target_t"][b].cpu().reshape(3)))
    return add, r, t
