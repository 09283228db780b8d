"""The CPU oracle against known answers (the reference ships no tests or golden vectors,
SURVEY.md §4): kNN on hand-checkable point sets, the tie rule, EPnP / RANSAC exact recovery,
bilinear conventions, and the state-dict contract shared with the product model."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import pnp
from oracle.krrn_oracle import KRRNOracle, get_nearest_index, get_neighbor_index
from pose_estimation_amd import KRRN, make_config

K4 = np.array([572.4114, 573.57043, 325.2611, 242.04899])


def test_knn_line_known_answer():
    # points on a line at x = 0, 1, 3, 7, 15: neighbours are unambiguous
    v = torch.tensor([[[0., 0, 0], [1, 0, 0], [3, 0, 0], [7, 0, 0], [15, 0, 0]]])
    idx = get_neighbor_index(v, 2)
    assert idx[0].tolist() == [[1, 2], [0, 2], [1, 0], [2, 1], [3, 2]]


def test_knn_tie_lower_index_wins():
    # query 0 at the origin, four candidates at distance 1 (indices 1..4): k=2 keeps 1, 2
    v = torch.tensor([[[0., 0, 0], [0, 1, 0], [1, 0, 0], [0, -1, 0], [-1, 0, 0]]])
    assert get_neighbor_index(v, 2)[0, 0].tolist() == [1, 2]
    # duplicates (wrap padding, batchdataset.py:680-685): "drop the first" drops the LOWER of
    # two coincident points, so point 2 keeps itself as its nearest neighbour
    v = torch.tensor([[[0., 0, 0], [5, 0, 0], [0, 0, 0]]])
    assert get_neighbor_index(v, 1)[0].tolist() == [[2], [0], [2]]


def test_nearest_known_answer():
    t = torch.tensor([[[0., 0, 0], [10, 0, 0], [4.9, 0, 0]]])
    s = torch.tensor([[[9., 0, 0], [1, 0, 0]]])
    assert get_nearest_index(t, s)[0, :, 0].tolist() == [1, 0, 1]


def _project(pw, R, t):
    pc = pw @ R.T + t
    return np.stack([K4[0] * pc[:, 0] / pc[:, 2] + K4[2], K4[1] * pc[:, 1] / pc[:, 2] + K4[3]], 1)


@pytest.mark.parametrize("n", [5, 6, 50, 256])
def test_epnp_exact_recovery(n):
    rng = np.random.default_rng(n)
    R = pnp.rotation_from_axis_angle(rng.normal(size=3))
    t = np.array([0.03, -0.05, 0.9])
    pw = rng.uniform(-0.06, 0.06, size=(n, 3))
    R2, t2, err = pnp.epnp(pw, _project(pw, R, t), K4)
    assert np.abs(R2 - R).max() < 1e-7 and np.abs(t2 - t).max() < 1e-7 and err < 1e-6


def test_epnp_planar_points():
    rng = np.random.default_rng(1)
    R = pnp.rotation_from_axis_angle([0.3, -0.2, 0.1])
    t = np.array([0.0, 0.0, 1.0])
    pw = np.concatenate([rng.uniform(-0.05, 0.05, size=(40, 2)), np.zeros((40, 1))], 1)
    R2, t2, _ = pnp.epnp(pw, _project(pw, R, t), K4)
    assert np.abs(R2 - R).max() < 1e-6 and np.abs(t2 - t).max() < 1e-6


def test_ransac_with_outliers_and_failure():
    rng = np.random.default_rng(2)
    R = pnp.rotation_from_axis_angle(rng.normal(size=3))
    t = np.array([0.05, 0.02, 0.8])
    pw = rng.uniform(-0.06, 0.06, size=(256, 3))
    uv = _project(pw, R, t)
    out = rng.random(256) < 0.25
    uv[out] += rng.uniform(10, 30, size=(out.sum(), 2)) * rng.choice([-1, 1], size=(out.sum(), 2))
    subs = np.stack([rng.choice(256, 5, replace=False) for _ in range(100)])
    R2, t2, cnt, mask, best = pnp.pnp_ransac(pw, uv, K4, subs)
    assert cnt == (~out).sum() and (mask == ~out).all()
    assert np.abs(R2 - R).max() < 1e-4 and np.abs(t2 - t).max() < 1e-4
    # pure noise: no hypothesis reaches 5 inliers -> failure, R = I, t = 0
    R3, t3, cnt3, _, best3 = pnp.pnp_ransac(pw, rng.uniform(0, 640, size=(256, 2)), K4, subs)
    assert cnt3 == 0 and best3 == -1 and np.allclose(R3, np.eye(3)) and np.all(t3 == 0)


def test_bilinear_conventions():
    # the HRNet fuse path uses align_corners=False, the heads align_corners=True
    x = torch.arange(16.).view(1, 1, 4, 4)
    a = F.interpolate(x, size=(8, 8), mode="bilinear", align_corners=False)
    b = torch.nn.UpsamplingBilinear2d(scale_factor=2.0)(x)
    assert a[0, 0, 0, 0] == 0 and b[0, 0, -1, -1] == 15 and not torch.equal(a, b)


@pytest.mark.parametrize("bb", ["w18", "w32", "lm"])
def test_state_dict_contract(bb):
    m = KRRN(cfg=make_config(num_cls=13, backbone=bb))
    o = KRRNOracle(num_cls=13, backbone=bb)
    a, b = m.state_dict(), o.state_dict()
    assert set(a) == set(b)
    assert all(a[k].shape == b[k].shape for k in a)
    # SURVEY.md §8b key families
    for k in ["backbone.conv1.weight", "backbone.layer1.0.downsample.1.running_var", "backbone.last_layer.0.0.bias",
              "backbone.last_layer.1.weight", "backbone.deconv_layer.0.0.weight", "backbone.deconv_layer.1.0.conv1.weight",
              "XYZNet.0.weight", "XYZNet.11.running_mean", "xyz_final.bias", "NMLNet.8.weight", "nml_final.weight",
              "fusion.conv_0_v.directions", "fusion.conv_1_x.weights", "fusion.bn2_n.running_var",
              "fusion.conv_4.directions", "fusion.conv_5.bias", "pose.t_net.conv1.weight", "pose.t_net.bn3.bias"]:
        assert k in a, k
    assert a["fusion.conv_4.directions"].shape == (9, 7 * 512)
    assert a["pose.t_net.conv1.weight"].shape == (1024, 1280 + 13, 1)
    assert a["xyz_final.weight"].shape[0] == (13 + 1) + 65 + 3 * 13
