"""pose_estimation_amd — MI355X-native KRRN dense-fusion inference path of
yaomy533/pose_estimation (HRNet + heads + 3D-GCN fusion + TBase + PnP-RANSAC), with every
arithmetic step in the gfx950 HIP library libkrrn_hip.so (include/krrn_hip.h).

Drop-in API (the reference's names):
    KRRN(num_cls, cfg)                    lib/network/krrn.py
    get_pose(pred, data)                  tools/trainer.py:383-438 (Trainer.get_pose)
    PoseDataset / make_batch              dataset/linemod/batchdataset.py (synthetic frames)
    Metric                                lib/utils/metric.py
    KRRNLoss                              lib/network/loss.py (eval-time terms)
"""
from .config import CONFIG, Cfg, make_config  # noqa: F401
from .krrn import KRRN  # noqa: F401
from .loss import KRRNLoss  # noqa: F401
from .pose import get_pose  # noqa: F401

__all__ = ["KRRN", "KRRNLoss", "get_pose", "make_config", "CONFIG", "Cfg"]
