"""Batched, sharded eval epoch: Trainer.test_epoch
(tools/trainer.py:145-250) over size-bucketed batches instead of one crop per step, split across
ranks.

Per batch of equal-size crops (BucketBatcher): the GPU-built inputs (PoseDataset.batch), one
KRRN forward, the eval-time KRRNLoss map terms per crop when the batch carries GT maps
(krrn_map_losses_crop_f32: the reference's batch-size-1 loop adds each crop's own losses,
trainer.py:180-182), get_pose (PnP-RANSAC, the "base" R / t), the TBase translation (the "reg" /
"final" t) and ADD(-S) / rotation / translation errors for the whole batch in one launch
(metric.cal_dis_batch). Each crop leaves one f64 record (REC fields below).

Multi-GPU (one process per GPU): every rank evaluates its own contiguous slice of every S bucket
(distributed.bucket_shard), the per-crop records are all-gathered (RCCL all_gather_into_tensor;
every rank knows every shard's size from the crop sizes, so records are padded to the largest
shard, no size exchange), and every rank folds them in global crop order — so the result dict,
sums included, is bit-identical for any world size. One all_reduce of the success counts checks
the gathered table against the ranks' own tallies.

The per-object bookkeeping keeps the reference's result keys and thresholds (ADD(-S) < 0.1 d,
5 deg, 5 cm); test_dis sums final ADD(-S) with opt_pose and base ADD(-S) without (:232-247);
the ADD(-S) AUC of Metric.cal_auc (metric.py:38-65) is reported per object and overall.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import distributed as kd
from .dataset import PoseDataset
from .krrn import KRRN
from .loss import map_losses
from .metric import Metric, add_metric, rt_errors
from .pose import get_pose

ROT_THR_DEG = 5.0     # trainer.py:156
TRANS_THR_M = 0.05    # trainer.py:157
_KEYS = ("all_num", "obj_num", "succ_base_rt", "dis_base_rt", "succ_base_r", "dis_base_r", "succ_base_t",
         "dis_base_t", "succ_reg_rt", "dis_reg_rt", "succ_reg_r", "dis_reg_r", "succ_reg_t", "dis_reg_t",
         "succ_final_rt", "dis_final_rt", "succ_final_r", "dis_final_r", "succ_final_t", "dis_final_t",
         "dis_mask", "dis_normal", "dis_xyz")
# per-crop record (f64)
REC = ("crop", "cls", "add_b", "r_b", "t_b", "add_f", "r_f", "t_f", "l_xyz", "l_mask", "l_normal", "valid")
_R = {k: i for i, k in enumerate(REC)}


def _batches(buckets: Dict[int, List[int]], bs: int):
    for S in sorted(buckets):
        idx = buckets[S]
        for lo in range(0, len(idx), bs):
            yield S, idx[lo:lo + bs]


@torch.no_grad()
def eval_records(model: KRRN, dataset: PoseDataset, indices: Dict[int, List[int]], bs: int, device,
                 opt_pose: bool = True, with_loss: bool = True) -> torch.Tensor:
    """Run the eval path over {S: [crop indices]} in batches of <= bs; returns f64 [n, len(REC)]
    (rows in the order evaluated). Every batch's inputs, forward, pose and ADD(-S) are queued on
    the device without a host round trip; the per-crop records are read back once at the end (the
    same numbers as a per-batch read-back, without a stall per batch).

    Three streams: batch j+1's inputs are built on one side stream while batch j's forward runs on
    the caller's stream (fresh tensors from resident frames), and batch j's PnP-RANSAC + ADD(-S)
    run on another beside batch j+1's forward (one workgroup per crop: latency-bound launches that
    fill the CUs the forward leaves idle). The pose reads a copy of the forward's 3-channel xyz map
    (the plan's buffer is rewritten by the next forward of the same shape). Host draws keep the
    serial order: forward j's pool perms, then get_pose j's point subsets, then forward j+1's."""
    metric = Metric(dataset.sym_obj)
    pending = []
    batches = list(_batches(indices, bs))
    device = torch.device(device)
    main = torch.cuda.current_stream(device)
    side = torch.cuda.Stream(device)   # inputs
    pstr = torch.cuda.Stream(device)   # pose + metric

    def build(j):
        side.wait_stream(main)  # the inputs' pinned staging and allocations follow earlier work
        with torch.cuda.stream(side):
            d = dataset.batch(batches[j][1], device)
            ev = torch.cuda.Event()
            ev.record(side)
        return d, ev

    nxt = build(0) if batches else None
    views = model.return_views
    model.return_views = True
    try:
        for j, (S, idx) in enumerate(batches):
            data, ev = nxt
            main.wait_event(ev)
            for v in data.values():
                v.record_stream(main)
                v.record_stream(pstr)
            if j + 1 < len(batches):
                nxt = build(j + 1)
            pred = model(data["img_croped"], data["cloud"], data["choose"], data["cls_id"], opt_pose=opt_pose)
            B = len(idx)
            lc = None
            if with_loss and "xyz" in data and "multi_cls_mask" in data:
                lc = map_losses(pred, data, per_crop=True)  # [B, 8]: xyz, normal, region, mask, counts
            # copies of what the pose step reads from the plan's output buffers
            xyz = pred["xyz"].clone()
            pred_t = pred["pred_t"].reshape(B, 3).clone() if opt_pose else None
            done = torch.cuda.Event()
            done.record(main)
            pstr.wait_event(done)
            xyz.record_stream(pstr)
            if pred_t is not None:
                pred_t.record_stream(pstr)
            with torch.cuda.stream(pstr):
                base_r, base_t = get_pose({"xyz": xyz}, data)
                add_b = add_metric(base_r, base_t.reshape(B, 3), data["model_points"], data["target"],
                                   data["cls_id"], metric.sys)
                add_f = None
                if opt_pose:
                    # reg = final = (PnP R, TBase t) (trainer.py:198-201)
                    add_f = add_metric(base_r, pred_t, data["model_points"], data["target"], data["cls_id"],
                                       metric.sys)
            pending.append((idx, data["cls_id"], data["target_r"], data["target_t"], base_r, base_t, pred_t, add_b,
                            add_f, lc))
    finally:
        model.return_views = views
    main.wait_stream(pstr)
    for p in pending:  # made on the pose stream, read back on the caller's
        for t in (p[4], p[5], p[7], p[8]):
            if t is not None:
                t.record_stream(main)
    if not pending:
        return torch.zeros((0, len(REC)), dtype=torch.float64)
    # one read-back and one vectorised host pass for the whole epoch: per batch, the rotation /
    # translation errors' six small copies and ~60 CPU ops ran after the GPU had drained (a serial
    # host tail of ~1 ms per batch); every quantity is per crop, so the values are the same
    cat = lambda k, w: torch.cat([p[k].reshape(len(p[0]), w) for p in pending])  # noqa: E731
    n = sum(len(p[0]) for p in pending)
    rec = np.zeros((n, len(REC)), dtype=np.float64)
    rec[:, _R["crop"]] = np.concatenate([np.asarray(p[0], dtype=np.float64) for p in pending])
    rec[:, _R["cls"]] = cat(1, 1).reshape(n).cpu().numpy()
    rec[:, _R["valid"]] = 1.0
    o = 0
    for p in pending:
        if p[9] is not None:
            lcn = p[9].cpu().numpy()
            rec[o:o + len(p[0]), _R["l_xyz"]] = lcn[:, 0]
            rec[o:o + len(p[0]), _R["l_normal"]] = lcn[:, 1]
            rec[o:o + len(p[0]), _R["l_mask"]] = lcn[:, 3]
        o += len(p[0])
    base_r, tr, tt = cat(4, 9), cat(2, 9), cat(3, 3)
    rec[:, _R["add_b"]] = cat(7, 1).reshape(n).cpu().numpy()
    rec[:, _R["r_b"]], rec[:, _R["t_b"]] = rt_errors(base_r, cat(5, 3), tr, tt)
    if opt_pose:
        rec[:, _R["add_f"]] = cat(8, 1).reshape(n).cpu().numpy()
        rec[:, _R["r_f"]], rec[:, _R["t_f"]] = rt_errors(base_r, cat(6, 3), tr, tt)
    return torch.from_numpy(rec)


def fold_records(records: torch.Tensor, objlist: Sequence[int], diameter: Sequence[float], opt_pose: bool,
                 metric: Metric) -> Dict[str, object]:
    """The reference's per-object bookkeeping (trainer.py:165-250) over per-crop records, in global
    crop order (independent of how crops were batched or sharded)."""
    rec = records.numpy() if isinstance(records, torch.Tensor) else np.asarray(records)
    rec = rec[rec[:, _R["valid"]] > 0]
    rec = rec[np.argsort(rec[:, _R["crop"]], kind="stable")]
    result = {k: {o: 0.0 for o in objlist} for k in _KEYS}
    cls = rec[:, _R["cls"]].astype(np.int64)
    col = lambda k: rec[:, _R[k]]  # noqa: E731

    def seq_sum(x):  # the reference's running `+=` in crop order (np.cumsum adds sequentially)
        return float(np.cumsum(x)[-1]) if len(x) else 0.0

    # first-appearance order of the objects, as the reference's dict of ADD lists fills
    order = [int(c) for c in dict.fromkeys(cls.tolist())]
    adds: Dict[int, List[float]] = {}
    for c in order:
        obj, dia = objlist[c], diameter[c]
        sel = cls == c
        n = float(sel.sum())
        result["all_num"][obj] = result["obj_num"][obj] = n
        ab, rb, tb = col("add_b")[sel], col("r_b")[sel], col("t_b")[sel]
        result["dis_base_rt"][obj] = seq_sum(ab)
        result["dis_base_r"][obj] = seq_sum(rb)
        result["dis_base_t"][obj] = seq_sum(tb)
        result["succ_base_rt"][obj] = float((ab < 0.1 * dia).sum())
        result["succ_base_r"][obj] = float((rb < ROT_THR_DEG).sum())
        result["succ_base_t"][obj] = float((tb < TRANS_THR_M).sum())
        result["dis_xyz"][obj] = seq_sum(col("l_xyz")[sel])
        result["dis_mask"][obj] = seq_sum(col("l_mask")[sel])
        result["dis_normal"][obj] = seq_sum(col("l_normal")[sel])
        if opt_pose:
            af, rf, tf = col("add_f")[sel], col("r_f")[sel], col("t_f")[sel]
            for k in ("reg", "final"):
                result[f"dis_{k}_rt"][obj] = seq_sum(af)
                result[f"dis_{k}_r"][obj] = seq_sum(rf)
                result[f"dis_{k}_t"][obj] = seq_sum(tf)
                result[f"succ_{k}_rt"][obj] = float((af < 0.1 * dia).sum())
                result[f"succ_{k}_r"][obj] = float((rf < ROT_THR_DEG).sum())
                result[f"succ_{k}_t"][obj] = float((tf < TRANS_THR_M).sum())
            adds[obj] = af.tolist()
        else:
            adds[obj] = ab.tolist()
    out = copy.copy(result)
    out["test_count"] = int(len(rec))
    out["test_dis"] = seq_sum(col("add_f") if opt_pose else col("add_b")) / max(len(rec), 1)
    out["auc"] = {o: metric.cal_auc(v) for o, v in adds.items()}
    out["auc_all"] = metric.cal_auc([a for v in adds.values() for a in v]) if adds else 0.0
    return out


def gather_epoch_records(local: torch.Tensor, shard_sizes: Sequence[int], device, group=None) -> torch.Tensor:
    """All-gather every rank's [n_r, len(REC)] records (padded to max(shard_sizes) rows, pad rows
    have valid = 0) -> all ranks' records, rank-major."""
    world = len(shard_sizes)
    if world == 1:
        return local
    m = max(shard_sizes)
    pad = torch.zeros((max(m, 1), len(REC)), dtype=torch.float64)
    pad[:local.shape[0]] = local
    backend = dist.get_backend(group)
    buf = pad.to(device) if backend == "nccl" else pad
    out = kd.gather_records(buf, group=group)
    return out.cpu()


@torch.no_grad()
def test_epoch(model: KRRN, dataset: PoseDataset, bs: int = 64, device=None, opt_pose: bool = True,
               criterion=None, world: Optional[int] = None, rank: Optional[int] = None,
               group=None) -> Dict[str, object]:
    """Trainer.test_epoch over `dataset`. world/rank default to the initialised process group
    (1/0 without one). `criterion` enables the per-crop map-loss terms (dis_xyz / dis_mask /
    dis_normal) when the batches carry GT maps; the reference always evaluates it (:167)."""
    device = torch.device(device) if device is not None else next(model.parameters()).device
    if world is None:
        world = dist.get_world_size(group) if dist.is_initialized() else 1
    if rank is None:
        rank = dist.get_rank(group) if dist.is_initialized() else 0
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    sizes = [dataset.crop_size(i) for i in range(len(dataset))]
    mine = kd.bucket_shard(sizes, world, rank)
    local = eval_records(model, dataset, mine, bs, device, opt_pose=opt_pose, with_loss=criterion is not None)
    shard_sizes = [sum(len(v) for v in kd.bucket_shard(sizes, world, r).values()) for r in range(world)]
    allrec = gather_epoch_records(local, shard_sizes, device, group) if world > 1 else local
    metric = Metric(dataset.sym_obj)
    out = fold_records(allrec, dataset.objlist, dataset.diameter, opt_pose, metric)
    if world > 1:
        # the ranks' own crop / success tallies, summed, must equal the gathered table's
        key = "add_f" if opt_pose else "add_b"
        dia = torch.tensor([dataset.diameter[int(c)] for c in local[:, _R["cls"]]], dtype=torch.float64)
        mine_t = torch.tensor([float(local.shape[0]), float((local[:, _R[key]] < 0.1 * dia).sum())],
                              dtype=torch.float64)
        t = mine_t.to(device) if dist.get_backend(group) == "nccl" else mine_t
        dist.all_reduce(t, group=group)
        tot = t.cpu()
        succ_key = "succ_final_rt" if opt_pose else "succ_base_rt"
        assert int(tot[0]) == out["test_count"], (tot, out["test_count"])
        assert int(tot[1]) == int(sum(out[succ_key].values())), (tot, out[succ_key])
    return out
