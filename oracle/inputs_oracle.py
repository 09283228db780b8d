"""ORACLE (test infrastructure only — imported by tests/, never by the product path).

numpy restatement of the per-sample input construction of PoseDataset._load_data
(dataset/linemod/batchdataset.py:603-771) for one crop, given the frame and the snapped box:
crop + /255 + ImageNet normalisation (:70, 722, 744), the point mask (:662-666), the wrap-padded
`choose` when the mask has at most N pixels (:667-679), and the full-frame maps + back-projected
cloud of a given `choose` (:712-721). Arithmetic follows the reference's dtypes: u8 / 255. in f64
then f32; the cloud in f32 (numpy 1.x value-based casting keeps the python/np scalars f32 there).
"""
import numpy as np

MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def crop_inputs(rgb, depth, mask_label, rmin, cmin, S, obj_mask=None):
    img = rgb[rmin:rmin + S, cmin:cmin + S] / 255.
    img = img.astype(np.float32).transpose(2, 0, 1)
    img = (img - MEAN[:, None, None]) / STD[:, None, None]
    d = depth[rmin:rmin + S, cmin:cmin + S]
    m = (mask_label[rmin:rmin + S, cmin:cmin + S] != 0) & (d != 0)
    if obj_mask is not None:
        m &= obj_mask[rmin:rmin + S, cmin:cmin + S] != 0
    return img.astype(np.float32), m


def choose_wrap(mask, N):
    ch = mask.flatten().nonzero()[0]
    assert 0 < len(ch) <= N
    return np.pad(ch, (0, N - len(ch)), "wrap")


def points(choose, depth, rmin, cmin, S, K4, depth_scale=1.0):
    fx, fy, cx, cy = [np.float32(v) for v in K4]
    r, c = choose // S, choose % S
    xm = (c + cmin).astype(np.float32)
    ym = (r + rmin).astype(np.float32)
    pt2 = depth[r + rmin, c + cmin].astype(np.float32) / np.float32(depth_scale)
    pt0 = (xm - cx) * pt2 / fx
    pt1 = (ym - cy) * pt2 / fy
    return np.stack([pt0, pt1, pt2], 1).astype(np.float32), xm, ym
