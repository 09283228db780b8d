"""Batched eval epoch: bucketed GPU-built batches through KRRN + get_pose +
Metric on a small synthetic LineMOD-all set; every crop is counted once, under its object."""
import pytest
import torch

from pose_estimation_amd import KRRN, make_config
from pose_estimation_amd.dataset import PoseDataset
from pose_estimation_amd.evaluate import test_epoch as run_epoch
from pose_estimation_amd.metric import Metric, cal_dis
from pose_estimation_amd.synthetic import init_weights

pytestmark = pytest.mark.gpu


def test_eval_epoch_counts(dev):
    ds = PoseDataset("test", 500, False, None, 0.0, 8, cls_type="all", num_frames=10, sizes=[80, 120, 80])
    m = KRRN(cfg=make_config(num_cls=len(ds.objlist), backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    res = run_epoch(m, ds, bs=4, device=dev)
    assert res["test_count"] == len(ds)
    assert sum(res["all_num"].values()) == len(ds)
    for o in ds.objlist:
        assert res["succ_final_rt"][o] <= res["all_num"][o]
    assert 0.0 <= res["auc_all"] <= 100.0


def test_eval_records_overlap_matches_serial(dev):
    """eval_records builds batch j+1's inputs on a side stream during batch j's forward and reads the
    model's output views in place: every record equals the plain serial loop's (fresh outputs, one
    stream), with the host and device RNG streams reset to the same state before each run."""
    import numpy as np
    from pose_estimation_amd import pose as kpose
    from pose_estimation_amd.evaluate import REC, _R, _batches, eval_records
    from pose_estimation_amd.metric import add_metric, rt_errors
    ds = PoseDataset("test", 500, False, None, 0.0, 8, cls_type="all", num_frames=14,
                     sizes=[80, 120, 80, 120, 80, 160, 80])
    m = KRRN(cfg=make_config(num_cls=len(ds.objlist), backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    buckets = {}
    for i in range(len(ds)):
        buckets.setdefault(ds.crop_size(i), []).append(i)
    metric = Metric(ds.sym_obj)

    def reset():
        torch.manual_seed(123)
        kpose._seeds.clear()
        ds._calls = 0

    reset()
    got = eval_records(m, ds, buckets, 3, dev, with_loss=False).numpy()
    reset()
    rows = []
    with torch.no_grad():
        for S, idx in _batches(buckets, 3):
            d = ds.batch(idx, dev)
            pred = m(d["img_croped"], d["cloud"], d["choose"], d["cls_id"])
            B = len(idx)
            br, bt = kpose.get_pose(pred, d)
            pt = pred["pred_t"].reshape(B, 3)
            add_b = add_metric(br, bt.reshape(B, 3), d["model_points"], d["target"], d["cls_id"], metric.sys)
            add_f = add_metric(br, pt, d["model_points"], d["target"], d["cls_id"], metric.sys)
            rec = np.zeros((B, len(REC)))
            rec[:, _R["crop"]] = idx
            rec[:, _R["cls"]] = d["cls_id"].reshape(B).cpu().numpy()
            rec[:, _R["valid"]] = 1.0
            rec[:, _R["add_b"]] = add_b.cpu().numpy()
            rec[:, _R["r_b"]], rec[:, _R["t_b"]] = rt_errors(br, bt, d["target_r"], d["target_t"])
            rec[:, _R["add_f"]] = add_f.cpu().numpy()
            rec[:, _R["r_f"]], rec[:, _R["t_f"]] = rt_errors(br, pt, d["target_r"], d["target_t"])
            rows.append(rec)
    want = np.concatenate(rows)
    assert got.shape == want.shape
    assert np.array_equal(got, want), np.abs(got - want).max(0)


def test_cal_dis_gt_pose_is_zero(dev):
    ds = PoseDataset("test", 500, False, None, 0.0, 8, cls_type="all", num_frames=9, sizes=[80])
    data = ds.batch(list(range(len(ds))), dev)
    metric = Metric(ds.sym_obj)
    for b in range(len(ds)):
        add, r, t = cal_dis(metric, data["target_r"], data["target_t"], data, b)
        # angular_distance clamps |q1.q2| to 1 - 1e-7 (metric.py:93-97): identical R reads 0.051 deg
        assert add < 1e-6 and r < 0.06 and t < 1e-6


def test_eval_epoch_linemod_tree(dev, tmp_path):
    """test_epoch over a LineMOD-layout tree on disk (PoseDataset(root=...)): frames decoded and
    staged per batch, inputs built on the GPU bit-exact vs the numpy oracle of _load_data on the
    decoded frames, every crop evaluated once."""
    import numpy as np
    from linemod_tree import write_tree
    from oracle import inputs_oracle as io
    write_tree(str(tmp_path), objs=(6,), per_obj=5, sizes=(80, 120))
    ds = PoseDataset("test", 500, False, str(tmp_path), 0.0, 8, cls_type="cat")
    idx = [i for i in range(len(ds)) if ds.crop_size(i) == 80]
    data = ds.batch(idx, dev)
    torch.cuda.synchronize()
    for b, i in enumerate(idx):
        rgb, depth, ml = ds.tree.read(i)
        rmin, rmax, cmin, cmax = ds.boxes[i]
        img, m = io.crop_inputs(rgb, depth, ml, rmin, cmin, rmax - rmin)
        assert np.array_equal(data["img_croped"][b].cpu().numpy(), img)
        assert np.array_equal(data["point_mask"][b, 0].cpu().numpy().astype(bool), m)
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    res = run_epoch(m, ds, bs=4, device=dev)
    assert res["test_count"] == len(ds) == 5
    assert res["all_num"][6] == 5


def test_eval_epoch_without_opt_pose(dev):
    """opt_pose=False: test_dis sums the base (PnP) ADD(-S) (trainer.py:245-247)."""
    ds = PoseDataset("test", 500, False, None, 0.0, 8, cls_type="all", num_frames=6, sizes=[80])
    m = KRRN(cfg=make_config(num_cls=len(ds.objlist), backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    res = run_epoch(m, ds, bs=4, device=dev, opt_pose=False)
    tot = sum(res["dis_base_rt"].values())
    assert res["test_dis"] > 0 and abs(res["test_dis"] - tot / len(ds)) < 1e-12
    assert sum(res["succ_final_rt"].values()) == 0
