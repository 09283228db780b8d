"""KRRNLoss at evaluation time (lib/network/loss.py:44-85), SURVEY.md §8f row f1.

tools/trainer.py:476 evaluates the criterion on every test batch, so the four dense map terms
(l1 on xyz, 1 - cosine on normals, cross-entropy on the region and mask logits, each over the
pixels whose target is non-zero — loss_utils.py:8-70) and the ADD(-S) PoseLoss (loss.py:19-42,
GT rotation with the predicted translation) run as two HIP launches each
(krrn_map_losses_f32, krrn_pose_loss_f32) instead of a chain of torch ops over the maps.

    crit = KRRNLoss(sym_list=SYM_OBJ, cfg=cfg)
    loss_dict = crit(pred, gt, opt_pose=True)     # same keys as the reference

The reference's `knn` argument (a KeOps argkmin, train.py:126) is accepted and ignored: the
nearest-target search is inside krrn_pose_loss_f32. Values are f64 device scalars.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Sequence

import torch

from . import _lib
from .config import CONFIG, SYM_OBJ
from .runtime import P, ptr

_I = ctypes.c_int
_L = ctypes.c_longlong
_lib.register("krrn_map_losses_ws", [_I, _I, P])
_lib.register("krrn_map_losses_f32", [P, P, P, P, P, _I, P, P, _I, P, _I, _I, P, P, P])
_lib.register("krrn_map_losses_crop_f32", [P, _I, _I, P, P])
_lib.register("krrn_pose_loss_ws", [_I, _I, P])
_lib.register("krrn_pose_loss_f32", [P, P, P, P, P, P, _I, _I, _I, P, P, P])


def _stream(dev) -> P:
    return P(torch.cuda.current_stream(dev).cuda_stream)


def _ws_size(fn: str, a: int, b: int) -> int:
    n = ctypes.c_longlong(0)
    _lib.check(getattr(_lib.lib(), fn)(a, b, ctypes.byref(n)), fn)
    return int(n.value)


def _f32(t: Optional[torch.Tensor], dev) -> Optional[torch.Tensor]:
    return None if t is None else t.to(device=dev, dtype=torch.float32).contiguous()


def _i64(t: Optional[torch.Tensor], dev) -> Optional[torch.Tensor]:
    return None if t is None else t.to(device=dev, dtype=torch.int64).contiguous()


def map_losses(pred: Dict[str, torch.Tensor], gt: Dict[str, torch.Tensor], per_crop: bool = False) -> torch.Tensor:
    """f64 [8]: l1(xyz), 1-cos(normal), CE(region), CE(mask), then the four valid-pixel counts
    (valid pixels pooled over the batch). per_crop=True: f64 [B, 8], each crop's own terms — what
    the reference's batch-size-1 test loop accumulates per object (trainer.py:180-182)."""
    xyz = pred["xyz"]
    dev = xyz.device
    if not xyz.is_cuda:
        raise RuntimeError("KRRNLoss runs on the HIP path only (pred maps must be GPU tensors)")
    B, _, H, W = xyz.shape
    HW = H * W
    region, mask = _f32(pred["region"], dev), _f32(pred["mask"], dev)
    region_gt = _i64(gt["region"].reshape(B, HW), dev)
    mask_gt = _i64(gt["multi_cls_mask"].reshape(B, HW), dev)
    ws = torch.empty(_ws_size("krrn_map_losses_ws", B, HW), dtype=torch.float64, device=dev)
    out = torch.empty(8, dtype=torch.float64, device=dev)
    _lib.call("krrn_map_losses_f32", ptr(_f32(xyz, dev)), ptr(_f32(gt["xyz"], dev)), ptr(_f32(pred["normal"], dev)),
              ptr(_f32(gt["normal"], dev)), ptr(region), region.shape[1], ptr(region_gt), ptr(mask), mask.shape[1],
              ptr(mask_gt), B, HW, ptr(ws), ptr(out), _stream(dev))
    if per_crop:
        oc = torch.empty((B, 8), dtype=torch.float64, device=dev)
        _lib.call("krrn_map_losses_crop_f32", ptr(ws), B, HW, ptr(oc), _stream(dev))
        return oc
    return out


def pose_loss(target_r: torch.Tensor, pred_t: torch.Tensor, target: torch.Tensor, model_points: torch.Tensor,
              cls_id: torch.Tensor, sym_list: Sequence[int]) -> torch.Tensor:
    """PoseLoss(pred_r=target_r, pred_t, targets, model_points, idxs) as KRRNLoss calls it."""
    dev = pred_t.device
    B, Pn = model_points.shape[0], model_points.shape[1]
    sym = torch.tensor(list(sym_list) or [0], dtype=torch.int32, device=dev)
    ws = torch.empty(_ws_size("krrn_pose_loss_ws", B, Pn), dtype=torch.float64, device=dev)
    out = torch.empty(1, dtype=torch.float64, device=dev)
    _lib.call("krrn_pose_loss_f32", ptr(_f32(target_r, dev)), ptr(_f32(pred_t.reshape(B, 3), dev)),
              ptr(_f32(target, dev)), ptr(_f32(model_points, dev)), ptr(_i64(cls_id.reshape(B), dev)), ptr(sym),
              len(sym_list), B, Pn, ptr(ws), ptr(out), _stream(dev))
    return out[0]


class KRRNLoss(torch.nn.Module):
    def __init__(self, sym_list: Sequence[int] = SYM_OBJ, knn=None, cfg=CONFIG):
        super().__init__()
        self.cfg = cfg
        self.sym_list = list(sym_list)
        self.loss_weight = cfg.Train.Loss.LOSS_WEIGHT

    def forward(self, pred, gt, opt_pose: bool = False):
        m = map_losses(pred, gt)
        loss_xyz, loss_normal, loss_region, loss_mask = m[0], m[1], m[2], m[3]
        if opt_pose:
            loss_add = pose_loss(gt["target_r"], pred["pred_t"], gt["target"], gt["model_points"], gt["cls_id"],
                                 self.sym_list)
        else:
            loss_add = 0
        w = self.loss_weight
        loss = (w["weight_xyz"] * loss_xyz + w["weight_region"] * loss_region + w["weight_mask"] * loss_mask
                + w["weight_normal"] * loss_normal + w["weight_pose"] * loss_add)
        return {"loss": loss, "loss_add": loss_add, "loss_xyz": loss_xyz, "loss_region": loss_region,
                "loss_normal": loss_normal, "loss_mask": loss_mask}
