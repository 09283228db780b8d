"""Pose-accuracy harness: Metric (lib/utils/metric.py:13-113) and Trainer.cal_dis
(tools/trainer.py:370-381) — the ADD(-S) / AUC half of BASELINE.json's metric.

ADD-S's nearest-prediction search (the reference broadcasts an [N, N, 3] tensor, metric.py:27-30)
runs on the HIP kNN kernel (krrn_knn_f32, mode 1, k = 1) when the points are on the GPU; the
distances of the selected pairs, means, quaternion angle and AUC are scalar bookkeeping.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .runtime import P, ptr


def _nearest_gpu(query: torch.Tensor, cand: torch.Tensor) -> torch.Tensor:
    """For each query row, the index of its nearest candidate (f32 expanded distance)."""
    q = query.contiguous().float()
    c = cand.contiguous().float()
    nq, nc = q.shape[0], c.shape[0]
    out = torch.empty((1, nq, 1), dtype=torch.int32, device=q.device)
    st = P(torch.cuda.current_stream(q.device).cuda_stream)
    _lib.check(_lib.lib().krrn_knn_f32(ptr(q), nq * 3, 3, nq, ptr(None), ptr(c), nc * 3, 3, nc, 3, 1, 0, 1, 1,
                                       ptr(out), st), "krrn_knn_f32")
    return out.view(nq).long()


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
        assert pred.dim() == target.dim() == 2
        add = float(torch.linalg.norm(pred - target, dim=1).mean())
        if idx in self.sys:
            if pred.is_cuda:
                nn = _nearest_gpu(target, pred)
                adds = float(torch.linalg.norm(target - pred[nn], dim=1).mean())
            else:  # host bookkeeping path for CPU tensors (harness only)
                d = torch.cdist(target.double(), pred.double())
                adds = float(d.min(dim=1)[0].mean())
            return adds, adds
        return add, add

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
        for i in range(1, prec.shape[0]):
            mpre[i] = max(mpre[i], mpre[i - 1])
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
