"""Micro-bench: krrn_pnp_ransac_f32 (get_pose, trainer.py:383-438) on a B = 64 batch of synthetic
scenes (exact model coordinates of a known pose, 10 % outliers, 0.4 px noise), H = 100.

usage (GPU box): python3 profiles/bench_pnp.py   (KRRN_HIP_LIB=build/variants/<v>.so for a variant)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import pose  # noqa: E402

dev = torch.device("cuda", 0)
B, N, S = int(os.environ.get("B", 64)), 1000, 120
K4 = np.array([572.4114, 573.57043, 325.2611, 242.04899], np.float32)
rng = np.random.default_rng(0)
ext = np.array([0.067, 0.1276, 0.1175])
lfb = np.array([-0.0335, -0.0638, -0.0587])
xyz = np.zeros((B, 3, S, S), np.float32)
choose = np.zeros((B, 1, N), np.int64)
xm = np.zeros((B, N, 1), np.float32)
ym = np.zeros((B, N, 1), np.float32)
for b in range(B):
    ax = rng.normal(size=3)
    th = np.linalg.norm(ax)
    k = ax / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    t = np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.7, 1.1)])
    pix = rng.choice(S * S, N, replace=False)
    u32 = rng.random((N, 3)).astype(np.float32)
    pc = (u32.astype(np.float64) * ext + lfb) @ R.T + t
    img = np.stack([K4[0] * pc[:, 0] / pc[:, 2] + K4[2], K4[1] * pc[:, 1] / pc[:, 2] + K4[3]], 1)
    img += rng.normal(scale=0.4, size=img.shape)
    out = rng.random(N) < 0.1
    img[out] += rng.uniform(-20, 20, size=(out.sum(), 2))
    xyz[b].reshape(3, -1)[:, pix] = u32.T
    choose[b, 0] = pix
    xm[b, :, 0], ym[b, :, 0] = img[:, 0], img[:, 1]
data = {"choose": torch.from_numpy(choose).to(dev), "x_map_choosed": torch.from_numpy(xm).to(dev),
        "y_map_choosed": torch.from_numpy(ym).to(dev), "intrinsic": torch.from_numpy(np.tile(K4, (B, 1))).to(dev),
        "extent": torch.from_numpy(np.tile(ext, (B, 1))).to(dev),
        "lfborder": torch.from_numpy(np.tile(lfb, (B, 1))).to(dev)}
pred = {"xyz": torch.from_numpy(xyz).to(dev)}
sel = pose.draw_sel(B, N, 256).to(dev)
_, _, info = pose.get_pose(pred, data, sel=sel, return_info=True)
subs = info["subsets"]


def run():
    return pose.get_pose(pred, data, sel=sel, subsets=subs, return_info=True)


for _ in range(3):
    run()
torch.cuda.synchronize()
a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    R, t, info = run()
b_.record()
torch.cuda.synchronize()
inl = info["inliers"].float()
print(f"B={B}: {a.elapsed_time(b_) / 20 * 1e3:8.1f} us per get_pose; inliers mean {inl.mean():.1f} "
      f"min {int(inl.min())}", flush=True)
