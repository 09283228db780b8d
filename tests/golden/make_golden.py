"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

Run from the repo root:  python tests/golden/make_golden.py

The reference cannot be imported or run here (import denied; it ships no tests
or stored outputs), so these vectors come from the oracle (oracle/krrn_oracle.py, a PyTorch-CPU
restatement of lib/network/krrn.py:27-165, and oracle/pnp_ref.c, the EPnP-RANSAC restatement
standing in for cv2.solvePnPRansac). They pin the oracle across rounds and give the GPU tests a
fixed target that does not need the oracle at run time. Weights are not stored: they are
re-derived from `init_weights(model, seed)` (torch CPU generator, deterministic).

Fixtures (.npz, float32 unless noted):
  krrn_cat_b1_s64_n256     C=1 'cat', HRNet-W18, B=1, S=64, N=256
  krrn_lm13_b2_s40_n128    C=13 LineMOD objlist, per-crop classes, B=2, S=40, N=128
                           (ragged GCN levels: N1=32, N2=8, k1=4, k2=1)
  pnp_scenes               get_pose KATs: clean, noisy, planar, pure-noise (failure)
  knn_lattice              kNN / nearest on integer-lattice points (massive distance ties)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import krrn_oracle as ko  # noqa: E402
from pose_estimation_amd.config import LM_OBJLIST, make_config  # noqa: E402
from pose_estimation_amd.fusion import level_sizes  # noqa: E402
from pose_estimation_amd.krrn import KRRN  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch, make_pnp_scene  # noqa: E402

KRRN_CASES = {
    # name: (num_cls, objlist, B, S, N, batch seed, weight seed, perm seed)
    "krrn_cat_b1_s64_n256": (1, None, 1, 64, 256, 7, 0, 3),
    "krrn_lm13_b2_s40_n128": (13, LM_OBJLIST, 2, 40, 128, 5, 1, 4),
}


def draw_perms(N: int, seed: int, k0: int = 10):
    """Pool_layer randperms in FusionNetLite call order (fusion.py:192-212)."""
    g = torch.Generator().manual_seed(seed)
    N1, N2, _, _ = level_sizes(N, k0)
    return [torch.randperm(N, generator=g)[:N1] for _ in range(4)] + [torch.randperm(N1, generator=g)[:N2]]


def krrn_case(num_cls, objlist, B, S, N, bseed, wseed, pseed):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    model = KRRN(cfg=make_config(num_cls=num_cls, backbone="w18"))
    sd = init_weights(model, wseed)
    o = ko.KRRNOracle(num_cls=num_cls, backbone="w18")
    o.load_state_dict(sd)
    o.eval()
    d = make_batch(B, S, N, seed=bseed, objlist=objlist)
    perms = draw_perms(N, pseed)
    tr = {}
    with torch.no_grad():
        out = o(d["img_croped"], d["cloud"], d["choose"], d["cls_id"], perms=perms, trace=tr)
    rec = {
        "img": d["img_croped"].numpy(), "cloud": d["cloud"].numpy(), "choose": d["choose"].numpy(),
        "cls": d["cls_id"].numpy(), "weight_seed": np.int64(wseed), "num_cls": np.int64(num_cls),
        "xyz": out["xyz"].numpy(), "normal": out["normal"].numpy(), "mask": out["mask"].numpy(),
        # region is R=65 channels at full res: keep a 4x-strided lattice of it
        "region_s4": out["region"][:, :, ::4, ::4].contiguous().numpy(),
        "pred_t": out["pred_t"].numpy(),
        "feat_s8": tr["feat"][:, ::8, :1280].contiguous().numpy(),
        # the pooled level-2 vertices the 9-D idx2 kNN runs on (tie justification of idx2 flips)
        "pool_2": tr["pool_2"].contiguous().numpy(),
    }
    for i, p in enumerate(perms):
        rec[f"perm{i}"] = p.numpy().astype(np.int32)
    for k in ("idx0", "idx1", "idx2", "nn1", "nn2"):
        rec[k] = tr[k].numpy().astype(np.int32)
    return rec


def pnp_case():
    scenes = [  # (seed, outlier_frac, noise_px, planar, pure_noise)
        (11, 0.1, 0.0, False, False),
        (12, 0.3, 0.4, False, False),
        (13, 0.1, 0.0, True, False),
        (14, 1.0, 0.0, False, True),
    ]
    B, N, S, P, H = 1, 300, 40, 256, 100
    rec = {}
    for i, (seed, of, nz, planar, noise) in enumerate(scenes):
        xyz, data, Rgt, tgt = make_pnp_scene(B, N, S, seed, outlier_frac=of, noise_px=nz, planar=planar)
        g = torch.Generator().manual_seed(seed)
        if noise:
            data["x_map_choosed"] = torch.rand(B, N, 1, generator=g) * 640
            data["y_map_choosed"] = torch.rand(B, N, 1, generator=g) * 480
        sel = torch.stack([torch.randperm(N, generator=g)[:P] for _ in range(B)]).int()
        subsets = torch.stack([torch.stack([torch.randperm(P, generator=g)[:5] for _ in range(H)])
                               for _ in range(B)]).int()
        R, t, cnt = ko.get_pose({"xyz": xyz}, data, sel, subsets)
        pre = f"s{i}_"
        rec.update({pre + "xyz": xyz.numpy(), pre + "choose": data["choose"].numpy(),
                    pre + "xmap": data["x_map_choosed"].numpy(), pre + "ymap": data["y_map_choosed"].numpy(),
                    pre + "intrinsic": data["intrinsic"].numpy(), pre + "extent": data["extent"].numpy(),
                    pre + "lfborder": data["lfborder"].numpy(), pre + "sel": sel.numpy(),
                    pre + "subsets": subsets.numpy(), pre + "R": R.numpy().astype(np.float32),
                    pre + "t": t.numpy().astype(np.float32), pre + "inliers": cnt.numpy().astype(np.int32),
                    pre + "R_gt": Rgt.astype(np.float32), pre + "t_gt": tgt.astype(np.float32)})
    rec["n_scenes"] = np.int64(len(scenes))
    return rec


def knn_case():
    rng = np.random.default_rng(21)
    # integer lattice coordinates: many exactly equal distances (tie -> lower index, the
    # stable topk the oracle pins), plus duplicated points (distance 0 to a non-self point)
    v = rng.integers(-3, 4, size=(2, 300, 3)).astype(np.float32)
    v[:, 7] = v[:, 3]
    v9 = np.concatenate([v, rng.integers(-2, 3, size=(2, 300, 6)).astype(np.float32)], 2)
    tv, t9 = torch.from_numpy(v), torch.from_numpy(v9)
    src = tv[:, ::4].contiguous()
    return {"v": v, "v9": v9,
            "idx_k10": ko.get_neighbor_index(tv, 10).numpy().astype(np.int32),
            "idx_k4": ko.get_neighbor_index(tv, 4).numpy().astype(np.int32),
            "idx9_k7": ko.get_neighbor_index(t9, 7).numpy().astype(np.int32),
            "nearest": ko.get_nearest_index(tv, src)[..., 0].numpy().astype(np.int32)}


def main():
    for name, args in KRRN_CASES.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **krrn_case(*args))
        print("wrote", name)
    np.savez_compressed(os.path.join(HERE, "pnp_scenes.npz"), **pnp_case())
    np.savez_compressed(os.path.join(HERE, "knn_lattice.npz"), **knn_case())
    print("wrote pnp_scenes, knn_lattice")


if __name__ == "__main__":
    main()
