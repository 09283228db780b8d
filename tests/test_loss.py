"""Eval-time KRRNLoss: the CPU oracle pinned by known answers, and the HIP
kernels (krrn_map_losses_f32, krrn_pose_loss_f32) against the oracle on identical inputs."""
import math

import pytest
import torch

from oracle import loss_oracle as lo
from pose_estimation_amd.config import SYM_OBJ


def _maps(B, H, W, R, M, seed):
    g = torch.Generator().manual_seed(seed)
    pred = {"xyz": torch.rand(B, 3, H, W, generator=g), "normal": torch.randn(B, 3, H, W, generator=g),
            "region": 3 * torch.randn(B, R, H, W, generator=g), "mask": 3 * torch.randn(B, M, H, W, generator=g)}
    valid = torch.rand(B, H, W, generator=g) < 0.6
    gt = {"xyz": torch.rand(B, 3, H, W, generator=g) * valid[:, None],
          "normal": torch.nn.functional.normalize(torch.randn(B, 3, H, W, generator=g), dim=1) * valid[:, None],
          "region": torch.randint(1, R, (B, H, W), generator=g) * valid,
          "multi_cls_mask": torch.randint(1, M, (B, H, W), generator=g) * valid}
    gt["normal"][0, :, 0, 0] = torch.tensor([0.0, 0.0, 1e-9])  # tiny non-zero target: eps clamp path
    return pred, gt


def _pose_inputs(B, P, seed, cls):
    g = torch.Generator().manual_seed(seed)
    mp = 0.05 * torch.randn(B, P, 3, generator=g)
    q = torch.nn.functional.normalize(torch.randn(B, 4, generator=g), dim=1)
    w, x, y, z = q.unbind(1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                     2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                     2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], 1).view(B, 3, 3)
    t = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 0.9])
    target = mp @ R.transpose(1, 2) + t[:, None]
    target = target[:, torch.randperm(P, generator=g)]  # order scrambled: only ADD-S recovers it
    pred_t = t + 0.01 * torch.randn(B, 3, generator=g)
    return R, pred_t, target, mp, torch.tensor(cls).view(B, 1)


def test_oracle_known_answers():
    B, R, H, W = 1, 5, 4, 4
    x = torch.zeros(B, R, H, W)
    lab = torch.full((B, 1, H, W), 2, dtype=torch.long)
    lab[..., 0, 0] = 0  # excluded pixel
    ce = lo.map_loss(lo.cross_entropy, x, lab)
    assert math.isclose(float(ce), -math.log(1.0 / R + 1e-6), rel_tol=1e-6)
    a = torch.ones(B, 3, H, W)
    t = torch.zeros(B, 3, H, W)
    t[:, :, :2] = 0.5
    assert math.isclose(float(lo.map_loss(lo.l1, a, t)), 1.5, rel_tol=1e-6)
    assert math.isclose(float(lo.map_loss(lo.cosine, t, t)), 0.0, abs_tol=1e-6)
    Rm, pt, tgt, mp, cls = _pose_inputs(2, 64, 0, [SYM_OBJ[0], 0])
    exact = lo.pose_loss(Rm, (tgt.mean(1) - (mp @ Rm.transpose(1, 2)).mean(1)).unsqueeze(1), tgt, mp,
                         cls.view(-1), SYM_OBJ)
    # crop 0 is symmetric: nearest matching undoes the scramble and the exact t gives ~0
    per = torch.norm(mp[0] @ Rm[0].T + (tgt[0].mean(0) - (mp[0] @ Rm[0].T).mean(0)) - tgt[0][lo.knn_nearest(
        mp[0] @ Rm[0].T + (tgt[0].mean(0) - (mp[0] @ Rm[0].T).mean(0)), tgt[0])], dim=1).mean()
    assert float(per) < 1e-6
    assert float(exact) > 0  # crop 1 keeps the scrambled correspondence


@pytest.mark.gpu
def test_map_losses_match_oracle(dev):
    from pose_estimation_amd.loss import map_losses
    pred, gt = _maps(2, 23, 17, 7, 4, seed=1)
    ref = lo.krrn_loss(pred, gt, SYM_OBJ, opt_pose=False)
    got = map_losses({k: v.to(dev) for k, v in pred.items()}, {k: v.to(dev) for k, v in gt.items()}).cpu()
    for i, k in enumerate(("loss_xyz", "loss_normal", "loss_region", "loss_mask")):
        assert math.isclose(float(got[i]), float(ref[k]), rel_tol=2e-6), (k, float(got[i]), float(ref[k]))
    valid = (gt["region"] != 0).sum()
    assert int(got[6]) == int(valid)


@pytest.mark.gpu
def test_pose_loss_match_oracle(dev):
    from pose_estimation_amd import KRRNLoss
    B, P = 3, 2600
    Rm, pt, tgt, mp, cls = _pose_inputs(B, P, 2, [SYM_OBJ[1], 3, SYM_OBJ[0]])
    ref = lo.pose_loss(Rm, pt.unsqueeze(1), tgt, mp, cls.view(-1), SYM_OBJ)
    crit = KRRNLoss(SYM_OBJ)
    pred, gt = _maps(B, 8, 8, 5, 3, seed=3)
    pred["pred_t"] = pt
    gt.update(target_r=Rm, target=tgt, model_points=mp, cls_id=cls)
    out = crit({k: v.to(dev) for k, v in pred.items()}, {k: v.to(dev) for k, v in gt.items()}, opt_pose=True)
    assert math.isclose(float(out["loss_add"]), float(ref), rel_tol=1e-5), (float(out["loss_add"]), float(ref))
    tot = sum(float(out[k]) for k in ("loss_xyz", "loss_region", "loss_mask", "loss_normal", "loss_add"))
    assert math.isclose(float(out["loss"]), tot, rel_tol=1e-12)


@pytest.mark.gpu
def test_map_losses_per_crop(dev):
    """Per-crop terms (the reference's batch-size-1 loop, trainer.py:180-182): crop b of a batch
    with different valid-pixel counts per crop equals the oracle run on crop b alone."""
    from pose_estimation_amd.loss import map_losses
    B = 3
    pred, gt = _maps(B, 31, 29, 7, 4, seed=5)
    for k in ("xyz", "normal"):
        gt[k][1, :, :20] = 0.0  # crop 1: far fewer valid pixels
    gt["region"][2, :25] = 0
    gt["multi_cls_mask"][0, :10] = 0
    got = map_losses({k: v.to(dev) for k, v in pred.items()}, {k: v.to(dev) for k, v in gt.items()}, per_crop=True).cpu()
    assert got.shape == (B, 8)
    for b in range(B):
        ref = lo.krrn_loss({k: v[b:b + 1] for k, v in pred.items()}, {k: v[b:b + 1] for k, v in gt.items()}, SYM_OBJ,
                           opt_pose=False)
        for i, k in enumerate(("loss_xyz", "loss_normal", "loss_region", "loss_mask")):
            assert math.isclose(float(got[b, i]), float(ref[k]), rel_tol=2e-6), (b, k, float(got[b, i]), float(ref[k]))
        assert int(got[b, 6]) == int((gt["region"][b] != 0).sum())
