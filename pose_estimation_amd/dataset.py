"""LineMOD-style eval loader with the per-sample work on the GPU (SURVEY.md §8b loader API,
§8f rows f2 and f3).

The reference's PoseDataset (dataset/linemod/batchdataset.py:34) reads one frame per item and
builds the crop in numpy (`_load_data`, :603-771): square-box snap, crop, ImageNet
normalisation, mask, random `choose`, back-projected cloud. Here the box snap stays on the host
(scalar integer logic, `get_square_bbox` below restates :890-961) and the per-pixel work runs for
a whole bucket of equal-size crops at once in two HIP launches (krrn_crop_inputs_u8,
krrn_choose_points). The frames live on the GPU.

`root` = a LineMOD tree in the reference's layout (Linemod_preprocessed): per object
`data/XX/{test,train}.txt` (image ids), `data/XX/gt.yml` (cam_R_m2c, cam_t_m2c in mm, obj_bb;
for benchvise the entry with obj_id 2, batchdataset.py:152-153, 229-240), `data/XX/rgb/NNNN.png`,
`data/XX/depth/NNNN.png` (uint16 mm), `data/XX/mask/NNNN.png` (mask_label = channel 0 == 255;
mode 'eval': `segnet_results/XX_label/NNNN_label.png` == 255, :197-244), and
`models/obj_XX.ply` (ascii PLY vertices / 1000, ply_vtx :841-852; 2600 random model points at
test time, :700-704). Only the crop sizes (from gt.yml's boxes) are read up front; each batch
reads and decodes its frames (a thread pool) and stages them to the GPU. Not read: the per-frame
GT-map pickles (xyz / normal / region, :202-212) — they feed only the logged loss terms and the
`mask_obj` factor of the point mask, so here the mask is mask_label * mask_depth (documented
deviation) and the loss keys are absent.

`root=None` (the default; no LineMOD data ships with the reference and there is no network)
serves seeded synthetic 640x480 RGB-D frames built like the real ones (an object mask inside a
YOLO-like detection box whose snapped sizes follow the LineMOD test histogram, a depth plane
with an object bump, LineMOD intrinsics and models_info extents, a GT pose and model points).

    ds = PoseDataset("test", 1000, False, None, 0.0, 8, cls_type="all")
    ds = PoseDataset("test", 1000, False, "/data/Linemod_preprocessed", 0.0, 8, cls_type="cat")
    for S, idx in BucketBatcher(ds, bs=64):      # f3: equal-S batches (trainer.py:521-551)
        data = ds.batch(idx, device)             # the eval keys of :730-771, on the GPU
"""
from __future__ import annotations

import ctypes
import os
import random
from collections import OrderedDict
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .config import CONFIG, LM_OBJLIST, OBJ_DICT, SYM_OBJ, models_info
from .runtime import P, h2d, ptr
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
    fi = h2d(torch.tensor(list(frame_idx), dtype=torch.int32), dev)
    rc = h2d(torch.tensor([[b[0], b[2]] for b in boxes], dtype=torch.int32), dev)
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
    K4 = h2d(K4, dev, torch.float32)
    _lib.call("krrn_choose_points", ptr(mask), B, S, N, ptr(depth), H, W, ptr(fi), ptr(rc), ptr(K4), float(depth_scale),
              ptr(seed), int(stream_id), ptr(choose), ptr(cloud), ptr(xm), ptr(ym), ptr(cnt), st)
    return {"img_croped": img, "choose": choose, "cloud": cloud, "x_map_choosed": xm, "y_map_choosed": ym,
            "point_mask": mask.view(B, 1, S, S), "mask_count": cnt}


def ply_vtx(path: str) -> np.ndarray:
    """Vertices of an ascii PLY (batchdataset.py:841-852: the element count on the 4th line, x y z
    the first three fields of each vertex line), f32 [n, 3] in the file's units."""
    with open(path) as f:
        if f.readline().strip() != "ply":
            raise ValueError(f"{path}: not a PLY file")
        n = None
        fmt = None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: no end_header")
            tok = line.split()
            if tok[:1] == ["format"]:
                fmt = tok[1]
            if tok[:2] == ["element", "vertex"]:
                n = int(tok[2])
            if line.strip() == "end_header":
                break
        if fmt != "ascii" or n is None:
            raise ValueError(f"{path}: only ascii PLY vertex lists are read (format {fmt})")
        return np.array([np.float32(f.readline().split()[:3]) for _ in range(n)], dtype=np.float32)


def _read_lines(p: str) -> List[str]:
    with open(p) as f:
        return [ln.strip() for ln in f if ln.strip()]


class _LinemodTree:
    """Index of a LineMOD tree (module doc): one entry per (object, image id) of the split, its GT
    pose and detection box from gt.yml; frames are read on demand."""

    def __init__(self, root: str, mode: str, objlist: Sequence[int], n_model_pts: int, seed: int):
        import yaml
        self.root, self.mode = root, mode
        self.items: List[Dict[str, object]] = []
        self.model_points: Dict[int, np.ndarray] = {}
        rng = np.random.default_rng(seed)
        split = "train.txt" if mode == "train" else "test.txt"
        for obj in objlist:
            croot = os.path.join(root, "data", f"{obj:02d}")
            with open(os.path.join(croot, "gt.yml")) as f:
                meta = yaml.safe_load(f)
            for im in _read_lines(os.path.join(croot, split)):
                entries = meta[int(im)]
                e = entries[0]
                if obj == 2:  # benchvise frames list several objects (batchdataset.py:230-234)
                    e = next((m for m in entries if int(m["obj_id"]) == 2), e)
                self.items.append({"obj": obj, "im": int(im), "R": np.resize(np.array(e["cam_R_m2c"], np.float64), (3, 3)),
                                   "t": np.array(e["cam_t_m2c"], np.float64) / 1000.0,
                                   "bbox": [float(v) for v in e["obj_bb"]]})
            pts = ply_vtx(os.path.join(root, "models", f"obj_{obj:02d}.ply")) / 1000.0
            if len(pts) < n_model_pts:
                # the reference's random.sample(range(len(pts)), len(pts) - num_pt_mesh_large) raises here
                # too (batchdataset.py:700-704): every crop's ADD(-S) runs over exactly n_model_pts points
                raise ValueError(f"obj_{obj:02d}.ply has {len(pts)} vertices < num_pt_mesh_large = {n_model_pts}")
            if len(pts) > n_model_pts:  # random deletion down to num_pt_mesh_large (:700-704)
                keep = np.sort(rng.choice(len(pts), n_model_pts, replace=False))
                pts = pts[keep]
            self.model_points[obj] = pts.astype(np.float32)

    def read(self, i: int):
        it = self.items[i]
        croot = os.path.join(self.root, "data", f"{int(it['obj']):02d}")
        im = int(it["im"])
        from PIL import Image
        with Image.open(os.path.join(croot, "rgb", f"{im:04d}.png")) as ri:
            rgb = np.array(ri)[:, :, :3]
        with Image.open(os.path.join(croot, "depth", f"{im:04d}.png")) as di:
            # depth / cam_scale (f64) then float32, as _load_data's depth_choosed (:714-716)
            depth = (np.asarray(di).astype(np.float64) / 1000.0).astype(np.float32)
        if self.mode == "eval":
            lp = os.path.join(self.root, "segnet_results", f"{int(it['obj']):02d}_label", f"{im:04d}_label.png")
        else:
            lp = os.path.join(croot, "mask", f"{im:04d}.png")
        with Image.open(lp) as li:
            label = np.array(li)
        ml = (label[:, :, 0] if label.ndim == 3 else label) == 255
        return rgb, depth, ml.astype(np.uint8)


class PoseDataset(torch.utils.data.Dataset):
    """The reference's constructor signature (batchdataset.py:34); `root` = a LineMOD tree, or
    None for synthetic frames (module doc). Eval only: add_noise / noise_trans / num_kps are
    accepted and unused."""

    def __init__(self, mode: str = "test", num_point: int = 1000, add_noise: bool = False, root: Optional[str] = None,
                 noise_trans: float = 0.0, num_kps: int = 8, cls_type: Optional[str] = None, cfg=CONFIG,
                 num_frames: int = 256, seed: int = 0, sizes: Optional[Sequence[int]] = None,
                 n_model_pts: int = 2600, io_threads: int = 8):
        self.mode, self.num_point, self.cfg, self.root = mode, num_point, cfg, root
        if cls_type in (None, "all"):
            self.objlist = list(LM_OBJLIST)
        else:
            self.objlist = [OBJ_DICT[cls_type]]
        self.sym_obj = [i for i in SYM_OBJ if i < len(self.objlist)] if len(self.objlist) > 1 else []
        info = models_info()
        self.diameter = [info[o]["diameter"] / 1000.0 for o in self.objlist]
        self.io_threads = io_threads
        if root is not None:
            self.tree = _LinemodTree(root, mode, self.objlist, n_model_pts, seed)
            self.frames_np = None
            self.boxes = [get_square_bbox(it["bbox"]) for it in self.tree.items]
        else:
            self.tree = None
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

    def _seed_for(self, device) -> torch.Tensor:
        key = str(device)
        if key not in self._seed:
            self._seed[key] = torch.tensor([int(np.random.SeedSequence(len(self)).generate_state(1)[0])],
                                           dtype=torch.int64, device=device)
        return self._seed[key]

    def frames(self, device) -> Dict[str, torch.Tensor]:
        """Synthetic frames, resident on `device` (all of them: 2.4 MB per 640x480 frame)."""
        key = str(device)
        if key not in self._dev_frames:
            self._dev_frames[key] = {k: torch.from_numpy(self.frames_np[k]).to(device)
                                     for k in ("rgb", "depth", "mask_label")}
        return self._dev_frames[key]

    def _read_frames(self, idx: Sequence[int], device) -> Dict[str, torch.Tensor]:
        """Decode the batch's frames from the tree (thread pool) and stage them on `device`."""
        with ThreadPoolExecutor(max_workers=max(1, min(self.io_threads, len(idx)))) as ex:
            fr = list(ex.map(self.tree.read, idx))
        return {"rgb": h2d(torch.from_numpy(np.stack([f[0] for f in fr])), device),
                "depth": h2d(torch.from_numpy(np.stack([f[1] for f in fr])), device),
                "mask_label": h2d(torch.from_numpy(np.stack([f[2] for f in fr])), device)}

    def _meta(self, i: int):
        """(obj id, R [3,3] f64, t [3] f64, model points [P,3] f32) of crop i."""
        if self.tree is not None:
            it = self.tree.items[i]
            obj = int(it["obj"])
            return obj, it["R"], it["t"], self.tree.model_points[obj]
        f = self.frames_np
        return (int(f["obj_id"][i]), f["target_r"][i].astype(np.float64), f["target_t"][i].astype(np.float64),
                f["model_points"][i])

    def batch(self, indices: Sequence[int], device) -> Dict[str, torch.Tensor]:
        """The eval keys of batchdataset.py:730-771 for `indices` (one crop size), collated."""
        device = torch.device(device)
        idx = list(indices)
        if self.tree is not None:
            fr = self._read_frames(idx, device)
            fidx = list(range(len(idx)))
        else:
            fr = self.frames(device)
            fidx = idx
        K4 = torch.tensor([[LM_K[0, 0], LM_K[1, 1], LM_K[0, 2], LM_K[1, 2]]] * len(idx), dtype=torch.float32)
        self._calls += 1
        out = build_inputs(fr, fidx, [self.boxes[i] for i in idx], self.num_point, K4, self._seed_for(device),
                           stream_id=self._calls)
        info = models_info()
        metas = [self._meta(i) for i in idx]
        ext = [np.array(info[m[0]]["size"]) / 1000.0 for m in metas]
        lfb = [np.array(info[m[0]]["min"]) / 1000.0 for m in metas]
        R64 = torch.from_numpy(np.stack([m[1] for m in metas]))
        t64 = torch.from_numpy(np.stack([m[2] for m in metas]))
        # every object keeps exactly num_pt_mesh_large model points (_LinemodTree / synthetic_frames), so
        # a batch mixing objects stacks them without cutting any crop's ADD(-S) point set
        assert len({len(m[3]) for m in metas}) == 1, [len(m[3]) for m in metas]
        mp = torch.from_numpy(np.stack([m[3] for m in metas]))
        host = {
            "cls_id": torch.tensor([[self.objlist.index(m[0])] for m in metas], dtype=torch.int64),
            "intrinsic": K4,
            "extent": torch.from_numpy(np.stack(ext)),
            "lfborder": torch.from_numpy(np.stack(lfb)),
            "bbox": torch.tensor([[b[0], b[1], b[2], b[3]] for b in (self.boxes[i] for i in idx)], dtype=torch.float32),
            "target_r": R64.float(), "target_t": t64.float(), "model_points": mp,
            # model_points @ target_r.T + target_t in f64, then float32 (batchdataset.py:706, 765)
            "target": (mp.double() @ R64.transpose(1, 2) + t64[:, None]).float(),
        }
        out.update({k: h2d(v, device) for k, v in host.items()})
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
