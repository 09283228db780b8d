"""HIP path (libkrrn_hip.so) vs the committed golden fixtures (tests/golden/make_golden.py):
no oracle at run time. Integer index work is bit-exact; float maps within MAP_RTOL of the
tensor's max magnitude; pred_t within T_ATOL metres."""
import ctypes
import os

import numpy as np
import pytest
import torch

from pose_estimation_amd import _lib, pose
from pose_estimation_amd.config import make_config
from pose_estimation_amd.krrn import KRRN
from pose_estimation_amd.runtime import P, ptr
from pose_estimation_amd.synthetic import init_weights
from tests.parity import knn_flips_at_ties

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAP_RTOL = 2e-4
T_ATOL = 1e-6       # pred_t when every discrete decision agrees with the fixture (north_star: 1e-3 mm)
T_ATOL_FLIP = 5e-5  # ... when a 9-D idx2 kNN entry flipped at a distance tie (justified below)


def _load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def _rel(a, ref):
    return float(np.abs(a - ref).max() / max(1e-12, np.abs(ref).max()))


@pytest.mark.parametrize("name", ["krrn_cat_b1_s64_n256", "krrn_lm13_b2_s40_n128"])
def test_krrn_golden(dev, name):
    g = _load(name)
    C = int(g["num_cls"])
    m = KRRN(cfg=make_config(num_cls=C, backbone="w18"))
    init_weights(m, int(g["weight_seed"]))
    m = m.to(dev).eval()
    m.keep_fusion_feat = True  # plan.feat is compared below
    t = lambda k: torch.from_numpy(g[k]).to(dev)  # noqa: E731
    perms = [t(f"perm{i}") for i in range(5)]
    out = m(t("img"), t("cloud"), t("choose"), t("cls"), perms=perms)
    torch.cuda.synchronize()
    for k in ("xyz", "normal", "mask"):
        assert _rel(out[k].cpu().numpy(), g[k]) < MAP_RTOL, k
    assert _rel(out["region"][:, :, ::4, ::4].cpu().numpy(), g["region_s4"]) < MAP_RTOL
    B, _, N = g["choose"].shape
    plan = m.get_plan(B, g["img"].shape[2], N, True)
    fb = plan.fusion_bufs
    for k in ("idx0", "idx1", "nn1", "nn2"):
        got = fb[k].cpu().numpy().reshape(g[k].shape)
        assert np.array_equal(got, g[k]), k
    # idx2 is decided on predicted (pooled 9-D) coordinates: an entry may differ only at a distance
    # tie within the coordinate perturbation + the kNN's own f32 rounding (tests/parity.py)
    n_bad, n_tie = knn_flips_at_ties(fb["idx2"].cpu().reshape(g["idx2"].shape), torch.from_numpy(g["idx2"]),
                                     fb["PV2"].cpu(), torch.from_numpy(g["pool_2"]), None, "idx2")
    assert n_bad == n_tie, (n_bad, n_tie)
    t_err = float(np.abs(out["pred_t"].cpu().numpy() - g["pred_t"]).max())
    print(f"pred_t |err| {t_err:.2e} m, idx2 flips at ties: {n_tie}")
    assert t_err < (T_ATOL if n_bad == 0 else T_ATOL_FLIP), t_err
    assert _rel(plan.feat[:, ::8].cpu().numpy(), g["feat_s8"]) < 5e-3


def _knn(q, c, k, drop, mode):
    B, nq, d = q.shape
    nc = c.shape[1]
    out = torch.empty((B, nq, k), dtype=torch.int32, device=q.device)
    st = P(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.lib().krrn_knn_f32(ptr(q), nq * d, d, nq, P(0), ptr(c), nc * d, d, nc, d, k, drop, mode, B,
                                       ptr(out), st), "krrn_knn_f32")
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_knn_golden(dev):
    g = _load("knn_lattice")
    v = torch.from_numpy(g["v"]).to(dev).contiguous()
    v9 = torch.from_numpy(g["v9"]).to(dev).contiguous()
    assert np.array_equal(_knn(v, v, 10, 1, 0), g["idx_k10"])
    assert np.array_equal(_knn(v, v, 4, 1, 0), g["idx_k4"])
    assert np.array_equal(_knn(v9, v9, 7, 1, 0), g["idx9_k7"])
    src = v[:, ::4].contiguous()
    assert np.array_equal(_knn(v, src, 1, 0, 1)[..., 0], g["nearest"])


def test_pnp_golden(dev):
    g = _load("pnp_scenes")
    for i in range(int(g["n_scenes"])):
        p = lambda k: torch.from_numpy(g[f"s{i}_{k}"])  # noqa: E731
        data = {"choose": p("choose"), "x_map_choosed": p("xmap"), "y_map_choosed": p("ymap"),
                "intrinsic": p("intrinsic"), "extent": p("extent"), "lfborder": p("lfborder")}
        R, t, info = pose.get_pose({"xyz": p("xyz").to(dev)}, data, num_points=g[f"s{i}_sel"].shape[1],
                                   sel=p("sel"), subsets=p("subsets"), return_info=True)
        torch.cuda.synchronize()
        cnt = int(info["inliers"][0])
        # the oracle restates the kernel's f64 expression order (oracle/pnp_ref.c): the same inlier
        # count and the pose to f32 rounding on every scene, the noisy one included
        assert cnt == int(g[f"s{i}_inliers"][0]), (i, cnt)
        assert np.abs(R.cpu().numpy() - g[f"s{i}_R"]).max() < 1e-6, i
        assert np.abs(t.cpu().numpy() - g[f"s{i}_t"]).max() < 1e-6, i
