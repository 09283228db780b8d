"""Seeded synthetic LineMOD-shaped inputs and weights.

No dataset or checkpoint ships with the reference and there is no network here, so the
benchmark and the parity tests run on synthetic crops built exactly like
PoseDataset._load_data builds real ones (dataset/linemod/batchdataset.py:603-771):
640x480 frame, LineMOD intrinsics, a square crop, an object mask, `choose` = N mask pixels
(wrap-padded when the mask is small, :673-687), depth back-projected to the camera-frame
`cloud` (:714-721), ImageNet-normalised RGB (:70, 744), extent / lfborder from
models_info.yml, and the GT pose / model points the metric needs.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from .config import LM_OBJLIST, OBJ_DICT, models_info

LM_K = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])
IMNET_MEAN = np.array([0.485, 0.456, 0.406], np.float32)
IMNET_STD = np.array([0.229, 0.224, 0.225], np.float32)


def rand_rotation(rng: np.random.Generator) -> np.ndarray:
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def make_batch(B: int, S: int, N: int, seed: int = 0, obj: str = "cat", objlist=None,
               frame=(480, 640), n_model_pts: int = 2600) -> Dict[str, torch.Tensor]:
    rng = np.random.default_rng(seed)
    H, W = frame
    info = models_info()
    objlist = objlist or [OBJ_DICT[obj]]
    fx, fy, cx, cy = LM_K[0, 0], LM_K[1, 1], LM_K[0, 2], LM_K[1, 2]
    out = {k: [] for k in ("img_croped", "cloud", "choose", "cls_id", "x_map_choosed", "y_map_choosed", "intrinsic",
                           "extent", "lfborder", "target_r", "target_t", "model_points", "target", "bbox", "mask")}
    yy, xx = np.mgrid[0:S, 0:S]
    for b in range(B):
        oid = objlist[b % len(objlist)] if len(objlist) > 1 else objlist[0]
        mi = info[oid]
        lf = np.array(mi["min"]) / 1000.0
        ext = np.array(mi["size"]) / 1000.0
        rmin = int(rng.integers(0, H - S + 1))
        cmin = int(rng.integers(0, W - S + 1))
        # object mask: an ellipse covering ~55% of the crop
        a, c = 0.42 * S, 0.42 * S
        m = (((yy - S / 2 + 0.5) / a) ** 2 + ((xx - S / 2 + 0.5) / c) ** 2) <= 1.0
        z0 = rng.uniform(0.7, 1.1)
        bump = 0.05 * np.sqrt(np.clip(1.0 - ((yy - S / 2) / a) ** 2 - ((xx - S / 2) / c) ** 2, 0, None))
        depth = (z0 - bump * m).astype(np.float32)
        ch = m.flatten().nonzero()[0]
        if len(ch) > N:
            sel = np.zeros(len(ch), dtype=int)
            sel[:N] = 1
            rng.shuffle(sel)
            ch = ch[sel.nonzero()]
        else:
            ch = np.pad(ch, (0, N - len(ch)), "wrap")
        xm = (xx + cmin).reshape(-1)[ch].astype(np.float32)
        ym = (yy + rmin).reshape(-1)[ch].astype(np.float32)
        dz = depth.reshape(-1)[ch]
        cloud = np.stack([(xm - cx) * dz / fx, (ym - cy) * dz / fy, dz], 1).astype(np.float32)
        img = rng.integers(0, 256, size=(S, S, 3)).astype(np.float32) / 255.0
        img = (img - IMNET_MEAN) / IMNET_STD
        R = rand_rotation(rng)
        t = np.array([((cmin + S / 2) - cx) * z0 / fx, ((rmin + S / 2) - cy) * z0 / fy, z0])
        mp = lf + rng.random((n_model_pts, 3)) * ext
        out["img_croped"].append(torch.from_numpy(img.transpose(2, 0, 1).copy()))
        out["cloud"].append(torch.from_numpy(cloud))
        out["choose"].append(torch.from_numpy(ch.astype(np.int64)).view(1, N))
        out["cls_id"].append(torch.tensor([objlist.index(oid) if len(objlist) > 1 else 0], dtype=torch.int64))
        out["x_map_choosed"].append(torch.from_numpy(xm).view(N, 1))
        out["y_map_choosed"].append(torch.from_numpy(ym).view(N, 1))
        out["intrinsic"].append(torch.tensor([fx, fy, cx, cy], dtype=torch.float32))
        out["extent"].append(torch.from_numpy(ext))
        out["lfborder"].append(torch.from_numpy(lf))
        out["target_r"].append(torch.from_numpy(R.astype(np.float32)))
        out["target_t"].append(torch.from_numpy(t.astype(np.float32)))
        out["model_points"].append(torch.from_numpy(mp.astype(np.float32)))
        out["target"].append(torch.from_numpy((mp @ R.T + t).astype(np.float32)))
        out["bbox"].append(torch.tensor([rmin, rmin + S, cmin, cmin + S], dtype=torch.float32))
        out["mask"].append(torch.from_numpy(m.astype(np.float32)).unsqueeze(0))
    return {k: torch.stack(v) for k, v in out.items()}


@torch.no_grad()
def init_weights(model: torch.nn.Module, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Deterministic random init of every parameter/buffer (keys in sorted order).

    conv / linear weights: normal, std = 0.7 / sqrt(fan_in) (measured to keep the W18 head
    outputs O(0.1) through the ~100-layer residual backbone; He gain sqrt(2) explodes to
    1e9 with random eval-BN statistics); biases 0.01 * randn; eval-BN gamma = 1 + 0.1 randn,
    beta = 0.1 randn, running_mean = 0.1 randn, running_var = U[0.5, 1.5];
    GCN weights / directions: the reference's uniform(-stdv, stdv) (gcn3d.py:84-86, 130-134).
    """
    g = torch.Generator().manual_seed(seed)
    sd = model.state_dict()
    out = {}
    for k in sorted(sd):
        v = sd[k]
        if v.dtype == torch.int64:
            out[k] = v.clone()
            continue
        leaf = k.rsplit(".", 1)[-1]
        shape = v.shape
        if leaf in ("weights", "directions"):
            cout = shape[1]
            stdv = 1.0 / math.sqrt(cout) if leaf == "weights" else 1.0 / math.sqrt(shape[1])
            t = (torch.rand(shape, generator=g) * 2 - 1) * stdv
        elif leaf == "bias" and k.rsplit(".", 2)[-2].startswith("conv_"):
            t = (torch.rand(shape, generator=g) * 2 - 1) / math.sqrt(shape[0])
        elif leaf == "running_var":
            t = 0.5 + torch.rand(shape, generator=g)
        elif leaf == "running_mean":
            t = 0.1 * torch.randn(shape, generator=g)
        elif leaf == "weight" and v.dim() == 1:  # BN gamma
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif leaf == "bias":
            t = (0.1 if _is_bn(k, sd) else 0.01) * torch.randn(shape, generator=g)
        elif leaf == "weight":
            if ".XYZNet.0." in f".{k}" or "deconv_layer.0.0" in k:
                fan_in = shape[0] * shape[2] * shape[3] / 4.0  # transposed conv: ~1/4 of taps per output
            else:
                fan_in = float(np.prod(shape[1:]))
            t = torch.randn(shape, generator=g) * (0.7 / math.sqrt(fan_in))
        else:
            t = torch.randn(shape, generator=g) * 0.02
        out[k] = t.to(v.dtype)
    model.load_state_dict(out)
    return out


def _is_bn(key: str, sd) -> bool:
    return key.rsplit(".", 1)[0] + ".running_mean" in sd


def make_pnp_scene(B: int, N: int, S: int, seed: int, outlier_frac: float = 0.1, noise_px: float = 0.0,
                   planar: bool = False):
    """get_pose inputs (trainer.py:383-438) whose chosen pixels hold the exact normalised
    model coordinates of a known pose: `xyz` [B,3,S,S], the data dict get_pose reads, and the
    ground truth (R [B,3,3], t [B,3]). Outliers are shifted by U[-20,20] px (SURVEY §8d KAT)."""
    rng = np.random.default_rng(seed)
    K4 = np.array([LM_K[0, 0], LM_K[1, 1], LM_K[0, 2], LM_K[1, 2]], np.float32)
    ext = np.array([0.067, 0.1276, 0.1175])
    lfb = np.array([-0.0335, -0.0638, -0.0587])
    xyz = np.zeros((B, 3, S, S), np.float32)
    choose = np.zeros((B, 1, N), np.int64)
    xm = np.zeros((B, N, 1), np.float32)
    ym = np.zeros((B, N, 1), np.float32)
    Rs, ts = [], []
    for b in range(B):
        R = rand_rotation(rng)
        t = np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.7, 1.1)])
        pix = rng.choice(S * S, N, replace=False)
        u32 = rng.random((N, 3)).astype(np.float32)
        if planar:
            u32[:, 2] = 0.5
        pw = u32.astype(np.float64) * ext + lfb
        pc = pw @ R.T + t
        img = np.stack([K4[0] * pc[:, 0] / pc[:, 2] + K4[2], K4[1] * pc[:, 1] / pc[:, 2] + K4[3]], 1)
        if noise_px:
            img += rng.normal(scale=noise_px, size=img.shape)
        out = rng.random(N) < outlier_frac
        img[out] += rng.uniform(-20, 20, size=(int(out.sum()), 2))
        xyz[b].reshape(3, -1)[:, pix] = u32.T
        choose[b, 0] = pix
        xm[b, :, 0] = img[:, 0]
        ym[b, :, 0] = img[:, 1]
        Rs.append(R)
        ts.append(t)
    data = {"choose": torch.from_numpy(choose), "x_map_choosed": torch.from_numpy(xm),
            "y_map_choosed": torch.from_numpy(ym), "intrinsic": torch.from_numpy(np.tile(K4, (B, 1))),
            "extent": torch.from_numpy(np.tile(ext, (B, 1))), "lfborder": torch.from_numpy(np.tile(lfb, (B, 1)))}
    return torch.from_numpy(xyz), data, np.stack(Rs), np.stack(ts)
