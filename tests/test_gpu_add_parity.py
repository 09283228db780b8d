"""BASELINE.json's accuracy criterion, "ADD(-S) within 0.1 % of the reference", at the metric layer.

Known-pose scenes (tests/test_gpu_pnp.py::_scene: chosen pixels hold the exact normalised model
coordinates of a known pose, 30 % outliers, optional pixel noise) go through the GPU get_pose and
through the C EPnP-RANSAC oracle on the GPU's selected subset (the subset choice itself is
chaotic on both sides, see test_gpu_pnp.py). Both poses are scored against the ground truth with
the reference's Metric (metric.py:17-65, Trainer.cal_dis trainer.py:370-381): ADD and ADD-S per
crop, the ADD(-S) < 0.1 d pass rate and the AUC (max_dis 0.1 m). The GPU numbers must agree with
the oracle's within 0.1 % (of the diameter per crop, and in AUC points) on noiseless scenes.

With 0.4 px noise the 5-point hypothesis of the selected subset carries the eigenvector-basis
ambiguity described in test_gpu_pnp.py at noise level; it moves correspondences sitting on the
1 px threshold in or out of the refinement set, which shifts single crops' refined poses by up to
a few mm of ADD (measured: 1 of 16 crops by 2.6 mm). There the pass rates must agree, single crops
within 5 % of the diameter, and the AUC within 0.5 points."""
import numpy as np
import pytest
import torch

from oracle import pnp as opnp
from pose_estimation_amd import pose
from pose_estimation_amd.metric import Metric

from test_gpu_pnp import K4, _cv2_select, _scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("noise_px", [0.0, 0.4])
def test_add_auc_matches_oracle(dev, noise_px):
    B, N, S = 16, 1000, 100
    xyz, data, Rgt, tgt = _scene(B, N, S, 3, outlier_frac=0.3, noise_px=noise_px)
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, return_info=True)
    torch.cuda.synchronize()
    sel = info["sel"].cpu().long()
    subs = info["subsets"].cpu()
    H = subs.shape[1]
    hcnt = info["workspace"].cpu()[B * H * 12:].view(torch.int32)[:B * H].view(B, H).numpy()
    ext = data["extent"][0].numpy()
    lfb = data["lfborder"][0].numpy()
    model = np.random.default_rng(5).random((500, 3)) * ext + lfb  # points of the object's box
    dia = float(np.linalg.norm(ext))
    metric = Metric(sym=[1])  # class 1 scored as symmetric (ADD-S), class 0 as ADD
    for cls in (0, 1):
        add_g, add_o = [], []
        for b in range(B):
            s = sel[b]
            pix = data["choose"][b, 0, s]
            obj = (xyz[b].reshape(3, -1)[:, pix].double().t() * data["extent"][b] + data["lfborder"][b]).float().numpy()
            img = np.stack([data["x_map_choosed"][b, s, 0].numpy(), data["y_map_choosed"][b, s, 0].numpy()], 1)
            best_h = _cv2_select(hcnt[b], len(s))
            Ro, to, _, _, _ = opnp.pnp_ransac(obj, img, K4, subs[b, best_h:best_h + 1].numpy(), 1.0)
            target = torch.from_numpy(model @ Rgt[b].T + tgt[b]).float().to(dev)
            pg = torch.from_numpy(model @ R[b].cpu().double().numpy().T + t[b].cpu().double().numpy()).float().to(dev)
            po = torch.from_numpy(model @ np.asarray(Ro, np.float64).T + np.asarray(to, np.float64)).float().to(dev)
            add_g.append(metric.cal_adds_cuda(pg, target, cls)[0])
            add_o.append(metric.cal_adds_cuda(po, target, cls)[0])
        add_g, add_o = np.array(add_g), np.array(add_o)
        crop_tol, auc_tol = (1e-3 * dia, 0.1) if noise_px == 0.0 else (5e-2 * dia, 0.5)
        assert np.abs(add_g - add_o).max() < crop_tol, (cls, np.abs(add_g - add_o).max())
        assert ((add_g < 0.1 * dia) == (add_o < 0.1 * dia)).all()
        auc_g, auc_o = metric.cal_auc(list(add_g)), metric.cal_auc(list(add_o))
        assert abs(auc_g - auc_o) < auc_tol, (cls, auc_g, auc_o)
        assert auc_g > 90.0  # the poses are recovered (AUC over max_dis = 0.1 m)
