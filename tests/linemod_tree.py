"""Writes a small LineMOD-layout tree (the reference's Linemod_preprocessed layout read by
dataset/linemod/batchdataset.py:34-244, 841-852) from seeded synthetic frames, with PIL / yaml:
data/XX/{test.txt, gt.yml, rgb/NNNN.png, depth/NNNN.png (uint16 mm), mask/NNNN.png (3-channel,
255 = object)}, segnet_results/XX_label/NNNN_label.png (1-channel), models/obj_XX.ply (ascii)."""
import os

import numpy as np
import yaml
from PIL import Image

from pose_estimation_amd.dataset import synthetic_frames


def write_tree(root, objs=(6, 2), per_obj=3, sizes=(80, 120, 80), seed=0, n_vertices=3000):
    """Returns {(obj, im_id): frame dict} of what was written (depth as the mm uint16 image)."""
    written = {}
    rng = np.random.default_rng(seed)
    for k, obj in enumerate(objs):
        fr = synthetic_frames(per_obj, seed=seed + k, objlist=[obj], sizes=list(sizes))
        croot = os.path.join(root, "data", f"{obj:02d}")
        for sub in ("rgb", "depth", "mask"):
            os.makedirs(os.path.join(croot, sub), exist_ok=True)
        os.makedirs(os.path.join(root, "segnet_results", f"{obj:02d}_label"), exist_ok=True)
        ids = [3 * i + 1 for i in range(per_obj)]
        meta = {}
        for f, im in enumerate(ids):
            Image.fromarray(fr["rgb"][f]).save(os.path.join(croot, "rgb", f"{im:04d}.png"))
            dmm = np.round(fr["depth"][f].astype(np.float64) * 1000.0).astype(np.uint16)
            Image.fromarray(dmm).save(os.path.join(croot, "depth", f"{im:04d}.png"))
            m = fr["mask_label"][f]
            Image.fromarray(np.stack([m, m, m], -1)).save(os.path.join(croot, "mask", f"{im:04d}.png"))
            Image.fromarray(m).save(os.path.join(root, "segnet_results", f"{obj:02d}_label", f"{im:04d}_label.png"))
            x, y, w, h = (int(round(v)) for v in fr["bbox"][f])
            entry = {"cam_R_m2c": [float(v) for v in fr["target_r"][f].reshape(-1)],
                     "cam_t_m2c": [float(v) * 1000.0 for v in fr["target_t"][f]], "obj_bb": [x, y, w, h],
                     "obj_id": obj}
            # benchvise frames list other objects first (the loader must pick obj_id 2)
            meta[im] = ([{"cam_R_m2c": [1.0, 0, 0, 0, 1, 0, 0, 0, 1], "cam_t_m2c": [0.0, 0.0, 1.0],
                          "obj_bb": [0, 0, 10, 10], "obj_id": 5}] if obj == 2 else []) + [entry]
            written[(obj, im)] = {"rgb": fr["rgb"][f], "depth_mm": dmm, "mask": m, "bbox": [x, y, w, h],
                                  "R": fr["target_r"][f], "t": fr["target_t"][f]}
        with open(os.path.join(croot, "gt.yml"), "w") as fh:
            yaml.safe_dump(meta, fh)
        with open(os.path.join(croot, "test.txt"), "w") as fh:
            fh.write("".join(f"{im:04d}\n" for im in ids))
        os.makedirs(os.path.join(root, "models"), exist_ok=True)
        v = (rng.random((n_vertices, 3)) - 0.5) * 100.0  # mm
        with open(os.path.join(root, "models", f"obj_{obj:02d}.ply"), "w") as fh:
            fh.write(f"ply\nformat ascii 1.0\nelement vertex {n_vertices}\nproperty float x\nproperty float y\n"
                     "property float z\nelement face 0\nproperty list uchar int vertex_indices\nend_header\n")
            fh.write("".join(f"{a:.4f} {b:.4f} {c:.4f}\n" for a, b, c in v))
    return written
