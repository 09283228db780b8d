"""KRRN configuration (the reference's mmcv `cfg.Module.* / cfg.Data.*` tree).

The reference loads `config/linemod/lm_v3_1.py`, which is an empty file in the repository
(SURVEY.md §0.2), so every value below is re-derived:

  Module.NUM_CLS           = C (len(objlist); KRRN.__init__ ignores its num_cls argument,
                             lib/network/krrn.py:27-30)
  Module.BACKBONE          = HRNet variant yaml (configs/hrnet_{w18,w32,lm}.yaml)
  Module.BACKBONE_OUTC     = 128   (C_b, unknown in the reference; proposed in SURVEY §8a)
  Module.XYZNet.HEADEN_FS  = 128, XYZNet.OUT_FS = 3 (krrn.py:105 views as 3 per class)
  Module.NMLNet.HEADEN_FS  = 128, NMLNet.OUT_FS = 3
  Module.MASKNet.OUT_FS    = 1     (C+1 mask logits, batchdataset.py:671)
  Module.REGIONNet.OUT_FS  = 65    (64 FPS regions + background, batchdataset.py:723-728)
  Module.GCN3D.GCN_N_NUM   = 10, GCN_SUP_NUM = 7 (comments at fusion.py:140-143)
  Module.POSENet.INC_R     = 1280 (FusionNetLite width, fusion.py:237), OUT_T = 3
  Data.NUM_POINTS          = 1000, Data.RESIZE = False
"""
from __future__ import annotations

import copy
import functools
import os
from typing import Any, Dict

import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))
CONFIG_DIR = os.path.join(_HERE, "configs")


class Cfg(dict):
    """A dict with attribute access (the subset of mmcv.Config the model constructors use)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return Cfg({k: copy.deepcopy(v, memo) for k, v in self.items()})


def _to_cfg(d: Any):
    if isinstance(d, dict):
        return Cfg({k: _to_cfg(v) for k, v in d.items()})
    if isinstance(d, list):
        return [_to_cfg(v) for v in d]
    return d


def load_hrnet_spec(name: str) -> Cfg:
    path = name if os.path.isabs(name) else os.path.join(CONFIG_DIR, name)
    if not path.endswith(".yaml"):
        path = os.path.join(CONFIG_DIR, f"hrnet_{name}.yaml")
    with open(path) as f:
        return _to_cfg(yaml.safe_load(f))


def make_config(num_cls: int = 1, backbone: str = "w18", num_points: int = 1000, backbone_outc: int = 128,
                head_fs: int = 128, region_out: int = 65, **overrides) -> Cfg:
    cfg = _to_cfg({
        "Module": {
            "NUM_CLS": num_cls,
            "BACKBONE": backbone,
            "BACKBONE_OUTC": backbone_outc,
            "XYZNet": {"HEADEN_FS": head_fs, "OUT_FS": 3},
            "NMLNet": {"HEADEN_FS": head_fs, "OUT_FS": 3},
            "MASKNet": {"OUT_FS": 1},
            "REGIONNet": {"OUT_FS": region_out},
            "GCN3D": {"GCN_N_NUM": 10, "GCN_SUP_NUM": 7},
            "POSENet": {"INC_R": 1280, "OUT_T": 3, "OUTC_R": 4},
        },
        "Data": {"NUM_POINTS": num_points, "RESIZE": False},
        # KRRNLoss weights (lib/network/loss.py:56, cfg.Train.Loss.LOSS_WEIGHT): the values are in
        # the empty config file too, so every term is weighted 1 unless overridden
        "Train": {"Loss": {"LOSS_WEIGHT": {"weight_xyz": 1.0, "weight_region": 1.0, "weight_mask": 1.0,
                                           "weight_normal": 1.0, "weight_pose": 1.0}}},
    })
    for k, v in overrides.items():
        node = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            node = node[p]
        node[parts[-1]] = v
    return cfg


CONFIG = make_config()

# LineMOD object table (dataset/linemod/batchdataset.py:35-43) and models_info.yml values
# (dataset/linemod/dataset_config/models_info.yml: mm, converted to m on use).
OBJ_DICT = {'ape': 1, 'benchvise': 2, 'bowl': 3, 'cam': 4, 'can': 5, 'cat': 6, 'cup': 7, 'driller': 8,
            'duck': 9, 'eggbox': 10, 'glue': 11, 'holepuncher': 12, 'iron': 13, 'lamp': 14, 'phone': 15}
LM_OBJLIST = [1, 2, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15]
SYM_OBJ = [7, 8]  # indices into objlist (eggbox, glue), batchdataset.py:76


@functools.lru_cache(maxsize=1)
def _models_info() -> Dict[int, Dict[str, float]]:
    with open(os.path.join(CONFIG_DIR, "models_info.yaml")) as f:
        return {int(k): v for k, v in yaml.safe_load(f).items()}


def models_info() -> Dict[int, Dict[str, float]]:
    """models_info.yaml (parsed once per process; a deep copy per call, so callers may edit it)."""
    return copy.deepcopy(_models_info())
