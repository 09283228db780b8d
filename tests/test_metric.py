"""Metric (lib/utils/metric.py:17-113, Trainer.cal_dis trainer.py:370-381).

CPU: hand-computed known answers for cal_auc / voc_ap (including the reference's quirks: the
recall axis closes at 0.1 and the area is scaled x10, the precision envelope loop runs over
indices 1..n-1 of mpre only) and for angular_distance (the |q1.q2| clamp at 1 - 1e-7 reads
0.0512 deg for identical rotations). GPU: the batched krrn_add_metric_f32 ADD / ADD-S against
the reference's own broadcast formula (norm of [N, N, 3] differences, min over predictions,
mean) on 2600-point sets, computed here with torch on the CPU."""
import math

import numpy as np
import pytest
import torch

from pose_estimation_amd.metric import Metric, rotation_matrix_to_quaternion


def test_cal_auc_known_answer():
    m = Metric([])
    # D -> [0.01, 0.02, 0.05, inf]; acc = [.25, .5, .75, 1]; mrec = [0, .01, .02, .05, .1],
    # mpre = [0, .25, .5, .75, .75]; area = .01*.25 + .01*.5 + .03*.75 + .05*.75 = .0675; x10 x100
    assert math.isclose(m.cal_auc([0.05, 0.01, 0.2, 0.02]), 67.5, rel_tol=1e-6)
    assert m.cal_auc([0.5, 0.2]) == 0  # nothing under max_dis
    # all at zero distance: area = 0.1 * 1 * 10 * 100
    assert math.isclose(m.cal_auc([0.0, 0.0, 0.0]), 100.0, rel_tol=1e-6)


def test_voc_ap_envelope_quirk():
    # prec = [.2, .1, .3]: the reference's loop lifts mpre[1..2] from mpre[i-1] only
    # (mpre = [0, .2, .2, .3, .3]); the areas of [0,.01,.02,.03,.1]
    rec = np.array([0.01, 0.02, 0.03])
    prec = np.array([0.2, 0.1, 0.3])
    want = (0.01 * 0.2 + 0.01 * 0.2 + 0.01 * 0.3 + 0.07 * 0.3) * 10
    assert math.isclose(Metric.voc_ap(rec, prec), want, rel_tol=1e-12)


def _rotz(deg):
    a = math.radians(deg)
    return torch.tensor([[math.cos(a), -math.sin(a), 0.0], [math.sin(a), math.cos(a), 0.0], [0.0, 0.0, 1.0]])


def test_angular_distance_known_answers():
    I = torch.eye(3).view(1, 3, 3)
    same = float(Metric.angular_distance(I, I))
    assert math.isclose(same, 2 * math.acos(1 - 1e-7) * 180 / math.pi, rel_tol=1e-9)  # 0.0512 deg
    for deg in (30.0, 90.0, 179.0):
        d = float(Metric.angular_distance(I, _rotz(deg).view(1, 3, 3)))
        assert abs(d - deg) < 1e-4, (deg, d)
    # q and -q are the same rotation (|q1.q2|): 190 deg about z reads as 170
    assert abs(float(Metric.angular_distance(I, _rotz(190.0).view(1, 3, 3))) - 170.0) < 1e-4


def test_quaternion_branches():
    """Shepperd's four branches (trace > 0, then the largest diagonal) give unit quaternions
    that rebuild the matrix."""
    g = torch.Generator().manual_seed(0)
    for R in [torch.eye(3), _rotz(179.0), torch.diag(torch.tensor([1.0, -1.0, -1.0])),
              torch.diag(torch.tensor([-1.0, 1.0, -1.0])), torch.diag(torch.tensor([-1.0, -1.0, 1.0]))] + \
             [torch.linalg.qr(torch.randn(3, 3, generator=g))[0] for _ in range(20)]:
        if torch.det(R) < 0:
            R = -R
        q = rotation_matrix_to_quaternion(R.double())
        w, x, y, z = q / q.norm()
        Rq = torch.tensor([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                           [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                           [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], dtype=torch.float64)
        assert torch.allclose(Rq, R.double(), atol=1e-6)


def _ref_adds(pred, target, sym):
    """metric.py:22-33 verbatim semantics (f32, CPU)."""
    add = torch.mean(torch.linalg.norm(pred - target, dim=1))
    if not sym:
        return float(add)
    N = pred.shape[0]
    pd = pred.view(1, N, 3).repeat(N, 1, 1)
    gt = target.view(N, 1, 3).repeat(1, N, 1)
    dis = torch.norm(pd - gt, dim=2)
    return float(torch.mean(torch.min(dis, dim=1)[0]))


@pytest.mark.gpu
def test_add_metric_vs_reference_broadcast(dev):
    from pose_estimation_amd.metric import add_metric
    B, P = 6, 2600
    g = torch.Generator().manual_seed(4)
    mp = (torch.rand(B, P, 3, generator=g) - 0.5) * 0.12
    Rs = torch.stack([torch.linalg.qr(torch.randn(3, 3, generator=g))[0] for _ in range(B)])
    Rs = Rs * torch.sign(torch.det(Rs)).view(B, 1, 1)
    t = torch.randn(B, 3, generator=g) * 0.05 + torch.tensor([0.0, 0.0, 0.9])
    tgt = mp @ Rs.transpose(1, 2) + t[:, None]
    # predicted pose: perturbed; targets scrambled for the symmetric crops
    Rp = Rs @ torch.stack([_rotz(3.0 * (b + 1)) for b in range(B)])
    tp = t + 0.003 * torch.randn(B, 3, generator=g)
    cls = torch.tensor([0, 1, 2, 1, 0, 1]).view(B, 1)
    sym = [1]
    for b in range(B):
        if int(cls[b]) in sym:
            tgt[b] = tgt[b][torch.randperm(P, generator=g)]
    got = add_metric(Rp.to(dev), tp.to(dev), mp.to(dev), tgt.to(dev), cls.to(dev), sym).cpu()
    for b in range(B):
        pred = mp[b] @ Rp[b].t() + tp[b]
        want = _ref_adds(pred, tgt[b], int(cls[b]) in sym)
        assert math.isclose(float(got[b]), want, rel_tol=2e-6), (b, float(got[b]), want)
    # Metric.cal_adds_cuda on already-transformed points (identity pose through the kernel)
    m = Metric(sym)
    pred = (mp[1] @ Rp[1].t() + tp[1]).to(dev)
    assert math.isclose(m.cal_adds_cuda(pred, tgt[1].to(dev), 1)[0], _ref_adds(pred.cpu(), tgt[1], True), rel_tol=2e-6)
