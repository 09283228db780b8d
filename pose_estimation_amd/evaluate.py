"""Batched eval epoch: Trainer.test_epoch (tools/trainer.py:145-250) over
size-bucketed batches instead of one crop per step.

Per batch of equal-size crops (BucketBatcher): the GPU-built inputs (PoseDataset.batch), one
KRRN forward, the eval-time KRRNLoss map terms when the batch carries GT maps, get_pose (PnP-
RANSAC, the "base" R / t) and the TBase translation (the "reg" / "final" t). The per-object
bookkeeping keeps the reference's result keys and thresholds (ADD(-S) < 0.1 d, 5 deg, 5 cm), and
the ADD(-S) AUC of Metric.cal_auc (metric.py:38-65) is reported per object and overall.
"""
from __future__ import annotations

import copy
from collections import defaultdict
from typing import Dict, Optional

import torch

from .dataset import BucketBatcher, PoseDataset
from .krrn import KRRN
from .loss import KRRNLoss
from .metric import Metric, cal_dis
from .pose import get_pose

ROT_THR_DEG = 5.0     # trainer.py:156
TRANS_THR_M = 0.05    # trainer.py:157
_KEYS = ("all_num", "obj_num", "succ_base_rt", "dis_base_rt", "succ_base_r", "dis_base_r", "succ_base_t",
         "dis_base_t", "succ_reg_rt", "dis_reg_rt", "succ_reg_r", "dis_reg_r", "succ_reg_t", "dis_reg_t",
         "succ_final_rt", "dis_final_rt", "succ_final_r", "dis_final_r", "succ_final_t", "dis_final_t",
         "dis_mask", "dis_normal", "dis_xyz")


@torch.no_grad()
def test_epoch(model: KRRN, dataset: PoseDataset, bs: int = 64, device=None, opt_pose: bool = True,
               criterion: Optional[KRRNLoss] = None) -> Dict[str, object]:
    device = torch.device(device) if device is not None else next(model.parameters()).device
    objlist = dataset.objlist
    metric = Metric(dataset.sym_obj)
    result = {k: {o: 0.0 for o in objlist} for k in _KEYS}
    adds = defaultdict(list)
    count, test_dis = 0, 0.0
    for S, idx in BucketBatcher(dataset, bs):
        data = dataset.batch(idx, device)
        pred = model(data["img_croped"], data["cloud"], data["choose"], data["cls_id"], opt_pose=opt_pose)
        losses = criterion(pred, data, opt_pose=False) if criterion is not None and "xyz" in data else None
        base_r, base_t = get_pose(pred, data)
        B = len(idx)
        for b in range(B):
            cls = int(data["cls_id"][b])
            obj = objlist[cls]
            dia = dataset.diameter[cls]
            result["all_num"][obj] += 1
            result["obj_num"][obj] += 1
            add, r, t = cal_dis(metric, base_r, base_t, data, b)
            result["dis_base_rt"][obj] += add
            result["dis_base_r"][obj] += r
            result["dis_base_t"][obj] += t
            result["succ_base_rt"][obj] += add < 0.1 * dia
            result["succ_base_r"][obj] += r < ROT_THR_DEG
            result["succ_base_t"][obj] += t < TRANS_THR_M
            if losses is not None:
                result["dis_xyz"][obj] += float(losses["loss_xyz"])
                result["dis_mask"][obj] += float(losses["loss_mask"])
                result["dis_normal"][obj] += float(losses["loss_normal"])
            if opt_pose:
                # reg = (PnP R, TBase t) = final (trainer.py:198-201)
                add, r, t = cal_dis(metric, base_r, pred["pred_t"], data, b)
                for k in ("reg", "final"):
                    result[f"dis_{k}_rt"][obj] += add
                    result[f"dis_{k}_r"][obj] += r
                    result[f"dis_{k}_t"][obj] += t
                    result[f"succ_{k}_rt"][obj] += add < 0.1 * dia
                    result[f"succ_{k}_r"][obj] += r < ROT_THR_DEG
                    result[f"succ_{k}_t"][obj] += t < TRANS_THR_M
                test_dis += add
            adds[obj].append(add)
            count += 1
    out = copy.copy(result)
    out["test_count"] = count
    out["test_dis"] = test_dis / max(count, 1)
    out["auc"] = {o: metric.cal_auc(v) for o, v in adds.items()}
    out["auc_all"] = metric.cal_auc([a for v in adds.values() for a in v])
    return out
