"""LineMOD-style eval loader with the per-sample work on the GPU (SURVEY.md §8b loader API,
§8f rows f2 and f3).

The reference's PoseDataset (dataset/linemod/batchdataset.py:34) reads one frame per item and
builds the crop in numpy (`_load_data`, :603-771): square-box snap, crop, ImageNet
normalisation, mask, random `choose`, back-projected cloud. Here the box snap stays on the host
(scalar integer logic, `get_square_bbox` below restates :890-961) and the per-pixel work runs for
a whole bucket of equal-size crops at once in two HIP launches (krrn_crop_inputs_u8,
krrn_choose_points). The frames live on the GPU.

No LineMOD data ships with the reference and there is no network, so `root=None` (the default)
serves seeded synthetic 640x480 RGB-D frames built like the real ones (an object mask inside a
YOLO-like detection box whose snapped sizes follow the LineMOD test histogram, a depth plane
with an object bump, LineMOD intrinsics and models_info extents, a GT pose and model points).

    ds = PoseDataset("test", 1000, False, None, 0.0, 8, cls_type="all")
    for S, idx in BucketBatcher(ds, bs=64):      # f3: equal-S batches (trainer.py:521-551)
        data = ds.batch(idx, device)             # the eval keys of :730-771, on the GPU
"""
from __future__ import annotations

import ctypes
import random
from collections import OrderedDict
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .config import CONFIG, LM_OBJLIST, OBJ_DICT, SYM_OBJ, models_info
from .runtime import P, ptr
from .synthetic import LM_K, rand_rotation

_I = ctypes.c_int
_F = ctypes.c_float
_lib.register("krrn_crop_inputs_u8", [P, P, P, P, _I, _I, _I, P, P, _I, _I, P, P, P])
_lib.register("krrn_choose_points", [P, _I, _I, _I, P, _I, _I, P, P, P, _F, P, _I, P, P, P, P, P, P])

# batchdataset.py:823
BORDER_LIST = [-1] + list(range(40, 640, 40)) + [640]
# measured LineMOD test crop sizes (get_square_bbox over bbox_yolov3_all.json)
LM_CROP_HIST = {40: 3, 80: 3025, 120: 4889, 160: 3659, 200: 1402, 240: 403, 280: 41, 320: 3}


def get_square_bbox(bbox, height_px: int = 480, width_px: int = 640) -> Tuple[int, int, int, int]:
    """batchdataset.py:890-961: [x, y, w, h] -> (rmin, rmax, cmin, cmax), a square whose side is
    snapped up to the 40-px border grid and shifted inside the frame."""
    bbx = [bbox[1], bbox[1] + bbox[3], bbox[0], bbox[0] + bbox[2]]
    if bbx[0] < 0:
        bbx[0] = 0
    if bbx[1] >= 480:
        bbx[1] = 479
    if bbx[2] < 0:
        bbx[2] = 0
    if bbx[3] >= 640:
        bbx[3] = 639
    rmin, rmax, cmin, cmax = bbx
    rmax += 1
    cmax += 1
    r_b = rmax - rmin
    c_b = cmax - cmin
    if r_b <= c_b:
        r_b = c_b
    else:
        c_b = r_b
    for tt in range(len(BORDER_LIST) - 1):
        if BORDER_LIST[tt] < r_b < BORDER_LIST[tt + 1]:
            r_b = BORDER_LIST[tt + 1]
            break
    for tt in range(len(BORDER_LIST) - 1):
        if BORDER_LIST[tt] < c_b < BORDER_LIST[tt + 1]:
            c_b = BORDER_LIST[tt + 1]
            break
    center = [int((rmin + rmax) / 2), int((cmin + cmax) / 2)]
    rmin = center[0] - int(r_b / 2)
    rmax = center[0] + int(r_b / 2)
    cmin = center[1] - int(c_b / 2)
    cmax = center[1] + int(c_b / 2)
    if rmin < 0:
        delt = -rmin
        rmin = 0
        rmax += delt
    if cmin < 0:
        delt = -cmin
        cmin = 0
        cmax += delt
    if rmax > height_px:
        delt = rmax - height_px
        rmax = height_px
        rmin -= delt
        if rmin < 0:
            rmax = rmax - rmin
            rmin = 0
            if rmax >= height_px:
                rmax = height_px - 1
    if cmax > width_px:
        delt = cmax - width_px
        cmax = width_px
        cmin -= delt
        if cmin < 0:
            cmax = cmax - cmin
            cmin = 0
            if cmax >= width_px:
                cmax = width_px - 1
    m = (rmax - rmin) - (cmax - cmin)
    if m > 0:
        rmax = rmax - np.floor(m / 2)
        rmin = rmin + np.floor(m / 2)
    elif m < 0:
        cmax = cmax + np.floor(m / 2)
        cmin = cmin - np.floor(m / 2)
    return int(rmin), int(rmax), int(cmin), int(cmax)


def synthetic_frames(F: int, seed: int = 0, objlist: Sequence[int] = (6,), H: int = 480, W: int = 640,
                     n_model_pts: int = 2600, sizes: Optional[Sequence[int]] = None) -> Dict[str, np.ndarray]:
    """Seeded full RGB-D frames with one object each (see module doc). Crop sizes are drawn from
    LM_CROP_HIST unless `sizes` fixes them (one per frame, cycled)."""
    rng = np.random.default_rng(seed)
    info = models_info()
    fx, fy, cx, cy = LM_K[0, 0], LM_K[1, 1], LM_K[0, 2], LM_K[1, 2]
    hs = np.array(list(LM_CROP_HIST.keys()))
    hp = np.array(list(LM_CROP_HIST.values()), dtype=np.float64)
    hp /= hp.sum()
    out = {k: [] for k in ("rgb", "depth", "mask_label", "bbox", "obj_id", "target_r", "target_t", "model_points")}
    yy, xx = np.mgrid[0:H, 0:W]
    for f in range(F):
        oid = objlist[f % len(objlist)]
        S = int(sizes[f % len(sizes)]) if sizes is not None else int(rng.choice(hs, p=hp))
        # a detection box whose snapped square is S (w, h in (S - 39, S - 1])
        w = S - 1 - rng.uniform(0.0, 30.0)
        h = S - 1 - rng.uniform(0.0, 30.0)
        x = rng.uniform(0, W - w - 1)
        y = rng.uniform(0, H - h - 1)
        ccy, ccx = y + h / 2, x + w / 2
        a, c = 0.45 * h, 0.45 * w
        m = (((yy - ccy) / a) ** 2 + ((xx - ccx) / c) ** 2) <= 1.0
        z0 = rng.uniform(0.7, 1.1)
        bump = 0.05 * np.sqrt(np.clip(1.0 - ((yy - ccy) / a) ** 2 - ((xx - ccx) / c) ** 2, 0, None))
        depth = (z0 - bump * m).astype(np.float32)
        depth[rng.random((H, W)) < 0.02] = 0.0  # sensor holes (mask_depth, :663)
        mi = info[oid]
        lf = np.array(mi["min"]) / 1000.0
        ext = np.array(mi["size"]) / 1000.0
        R = rand_rotation(rng)
        t = np.array([(ccx - cx) * z0 / fx, (ccy - cy) * z0 / fy, z0])
        out["rgb"].append(rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8))
        out["depth"].append(depth)
        out["mask_label"].append((m * 255).astype(np.uint8))
        out["bbox"].append(np.array([x, y, w, h], np.float32))
        out["obj_id"].append(oid)
        out["target_r"].append(R.astype(np.float32))
        out["target_t"].append(t.astype(np.float32))
        out["model_points"].append((lf + rng.random((n_model_pts, 3)) * ext).astype(np.float32))
    return {k: np.stack(v) for k, v in out.items()}


def build_inputs(frames: Dict[str, torch.Tensor], frame_idx: Sequence[int], boxes: Sequence[Tuple[int, int, int, int]],
                 num_point: int, K4: torch.Tensor, seed: torch.Tensor, stream_id: int = 0,
                 depth_scale: float = 1.0, obj_mask: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """The per-pixel half of _load_data for crops of one size on the GPU: img_croped, choose,
    cloud, x/y_map_choosed, plus the point mask and its pixel count per crop."""
    rgb, depth, ml = frames["rgb"], frames["depth"], frames["mask_label"]
    dev = rgb.device
    F, H, W = depth.shape
    B = len(frame_idx)
    sizes = {rmax - rmin for rmin, rmax, _, _ in boxes} | {cmax - cmin for _, _, cmin, cmax in boxes}
    if len(sizes) != 1:
        raise ValueError(f"one crop size per batch (bucket by get_square_bbox first), got {sorted(sizes)}")
    S = sizes.pop()
    fi = torch.tensor(list(frame_idx), dtype=torch.int32).to(dev)
    rc = torch.tensor([[b[0], b[2]] for b in boxes], dtype=torch.int32).to(dev)
    img = torch.empty((B, 3, S, S), dtype=torch.float32, device=dev)
    mask = torch.empty((B, S * S), dtype=torch.uint8, device=dev)
    st = P(torch.cuda.current_stream(dev).cuda_stream)
    _lib.call("krrn_crop_inputs_u8", ptr(rgb), ptr(depth), ptr(ml), ptr(obj_mask), F, H, W, ptr(fi), ptr(rc), B, S,
              ptr(img), ptr(mask), st)
    N = num_point
    choose = torch.empty((B, 1, N), dtype=torch.int64, device=dev)
    cloud = torch.empty((B, N, 3), dtype=torch.float32, device=dev)
    xm = torch.empty((B, N, 1), dtype=torch.float32, device=dev)
    ym = torch.empty((B, N, 1), dtype=torch.float32, device=dev)
    cnt = torch.empty((B,), dtype=torch.int32, device=dev)
    K4 = K4.to(device=dev, dtype=torch.float32).contiguous()
    _lib.call("krrn_choose_points", ptr(mask), B, S, N, ptr(depth), H, W, ptr(fi), ptr(rc), ptr(K4), float(depth_scale),
              ptr(seed), int(stream_id), ptr(choose), ptr(cloud), ptr(xm), ptr(ym), ptr(cnt), st)
    return {"img_croped": img, "choose": choose, "cloud": cloud, "x_map_choosed": xm, "y_map_choosed": ym,
            "point_mask": mask.view(B, 1, S, S), "mask_count": cnt}


class PoseDataset(torch.utils.data.Dataset):
    """The reference's constructor signature (batchdataset.py:34); root=None serves synthetic
    frames (module doc). Eval only: add_noise / noise_trans / num_kps are accepted and unused."""

    def __init__(self, mode: str = "test", num_point: int = 1000, add_noise: bool = False, root: Optional[str] = None,
                 noise_trans: float = 0.0, num_kps: int = 8, cls_type: Optional[str] = None, cfg=CONFIG,
                 num_frames: int = 256, seed: int = 0, sizes: Optional[Sequence[int]] = None):
        if root is not None:
            raise NotImplementedError("no LineMOD data ships with the reference; root=None serves synthetic frames")
        self.mode, self.num_point, self.cfg = mode, num_point, cfg
        if cls_type in (None, "all"):
            self.objlist = list(LM_OBJLIST)
        else:
            self.objlist = [OBJ_DICT[cls_type]]
        self.sym_obj = [i for i in SYM_OBJ if i < len(self.objlist)] if len(self.objlist) > 1 else []
        info = models_info()
        self.diameter = [info[o]["diameter"] / 1000.0 for o in self.objlist]
        self.frames_np = synthetic_frames(num_frames, seed, self.objlist, sizes=sizes)
        self.boxes = [get_square_bbox([float(v) for v in bb]) for bb in self.frames_np["bbox"]]
        self._dev_frames: Dict[str, Dict[str, torch.Tensor]] = {}
        self._seed: Dict[str, torch.Tensor] = {}
        self._calls = 0

    def __len__(self):
        return len(self.boxes)

    def crop_size(self, i: int) -> int:
        rmin, rmax, _, _ = self.boxes[i]
        return rmax - rmin

    def frames(self, device) -> Dict[str, torch.Tensor]:
        key = str(device)
        if key not in self._dev_frames:
            self._dev_frames[key] = {k: torch.from_numpy(self.frames_np[k]).to(device)
                                     for k in ("rgb", "depth", "mask_label")}
            self._seed[key] = torch.tensor([int(np.random.SeedSequence(len(self)).generate_state(1)[0])],
                                           dtype=torch.int64, device=device)
        return self._dev_frames[key]

    def batch(self, indices: Sequence[int], device) -> Dict[str, torch.Tensor]:
        """The eval keys of batchdataset.py:730-771 for `indices` (one crop size), collated."""
        device = torch.device(device)
        fr = self.frames(device)
        fnp = self.frames_np
        idx = list(indices)
        K4 = torch.tensor([[LM_K[0, 0], LM_K[1, 1], LM_K[0, 2], LM_K[1, 2]]] * len(idx), dtype=torch.float32)
        self._calls += 1
        out = build_inputs(fr, idx, [self.boxes[i] for i in idx], self.num_point, K4, self._seed[str(device)],
                           stream_id=self._calls)
        info = models_info()
        ext = [np.array(info[fnp["obj_id"][i]]["size"]) / 1000.0 for i in idx]
        lfb = [np.array(info[fnp["obj_id"][i]]["min"]) / 1000.0 for i in idx]
        R = torch.from_numpy(fnp["target_r"][idx])
        t = torch.from_numpy(fnp["target_t"][idx])
        mp = torch.from_numpy(fnp["model_points"][idx])
        host = {
            "cls_id": torch.tensor([[self.objlist.index(int(fnp["obj_id"][i]))] for i in idx], dtype=torch.int64),
            "intrinsic": K4,
            "extent": torch.from_numpy(np.stack(ext)),
            "lfborder": torch.from_numpy(np.stack(lfb)),
            "bbox": torch.tensor([[b[0], b[1], b[2], b[3]] for b in (self.boxes[i] for i in idx)], dtype=torch.float32),
            "target_r": R, "target_t": t, "model_points": mp,
            "target": (mp @ R.transpose(1, 2) + t[:, None]).float(),
        }
        out.update({k: v.to(device) for k, v in host.items()})
        return out

    def __getitem__(self, i: int) -> Dict[str, torch.Tensor]:
        dev = torch.device("cuda", torch.cuda.current_device())
        return {k: v[0].cpu() for k, v in self.batch([i], dev).items()}


class BucketBatcher:
    """Size-bucketed eval batches: the reference's process_patch_datas
    (tools/trainer.py:521-551) accumulates crops per square size and emits a batch of `bs` from a
    bucket holding more than `bs`; here every bucket is drained in `bs`-sized batches (the last
    one short) so each crop is evaluated exactly once, in dataset order within a bucket.
    Yields (S, [indices])."""

    def __init__(self, dataset: PoseDataset, bs: int, shuffle_buckets: bool = False, seed: int = 0):
        self.ds, self.bs = dataset, bs
        self.shuffle_buckets, self.seed = shuffle_buckets, seed

    def buckets(self) -> "OrderedDict[int, List[int]]":
        b: "OrderedDict[int, List[int]]" = OrderedDict()
        for i in range(len(self.ds)):
            b.setdefault(self.ds.crop_size(i), []).append(i)
        return OrderedDict(sorted(b.items()))

    def __iter__(self) -> Iterator[Tuple[int, List[int]]]:
        batches = []
        for S, idx in self.buckets().items():
            for lo in range(0, len(idx), self.bs):
                batches.append((S, idx[lo:lo + self.bs]))
        if self.shuffle_buckets:
            random.Random(self.seed).shuffle(batches)
        return iter(batches)

    def __len__(self):
        return sum((len(v) + self.bs - 1) // self.bs for v in self.buckets().values())
