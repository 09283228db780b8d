"""pose_estimation_amd — MI355X-native KRRN dense-fusion inference path of
yaomy533/pose_estimation (HRNet + heads + 3D-GCN fusion + TBase + PnP-RANSAC), with every
arithmetic step in the gfx950 HIP library libkrrn_hip.so (include/krrn_hip.h).

Drop-in API (the reference's names):
    KRRN(num_cls, cfg)                    lib/network/krrn.py
    get_pose(pred, data)                  tools/trainer.py:383-438 (Trainer.get_pose)
    PoseDataset / make_batch              dataset/linemod/batchdataset.py (synthetic frames)
    Metric                                lib/utils/metric.py
    KRRNLoss                              lib/network/loss.py (eval-time terms)
    dataset.PoseDataset / BucketBatcher   dataset/linemod/batchdataset.py + trainer.py:521-551
    evaluate.test_epoch                   tools/trainer.py:145-250 (batched)
    fps.farthest_point_sampling           tools/script/sample_model.py:35-48
    bpnp.BPnP / bpnp.BPnPModle            lib/network/dnn/BPnP.py (forward LM + implicit backward)
"""
from .config import CONFIG, Cfg, make_config  # noqa: F401
from .krrn import KRRN  # noqa: F401
from . import bpnp, dataset, fps  # noqa: F401  (register their C-ABI signatures)
from .loss import KRRNLoss  # noqa: F401
from .pose import get_pose  # noqa: F401

__all__ = ["KRRN", "KRRNLoss", "get_pose", "make_config", "CONFIG", "Cfg"]
