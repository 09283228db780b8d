"""Every environment variable the package reads, declared once (name -> default, meaning).

The defaults are the shipped configuration; each knob selects a measured alternative that still
exists in the code (for A/B timing on the GPU box, DESIGN.md records the numbers) or sizes a
cache. The C-ABI library reads no environment at all: its tuning is fixed at build time.
Modules read knobs at import time through `flag` / `integer` / `text`, so a value must be set
before the package is imported. tests/test_knobs.py checks that nothing outside this table is read.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

KNOBS: Dict[str, Tuple[Optional[str], str]] = {
    # --- loading, execution, capacity
    "KRRN_HIP_LIB": (None, "path of the C-ABI library to load instead of the in-tree libkrrn_hip.so "
                           "(variant builds for A/B timing, the KRRN_DIAG diagnostics build)"),
    "KRRN_GRAPH": ("1", "KRRN.forward replays a captured hipGraph of its plan; 0 = serial eager runs"),
    "KRRN_PLAN_STREAMS": ("1", "captured plans keep their side streams as graph branches; 0 = captured serially"),
    "KRRN_STREAMS": ("1", "the two-slot pipeline's stages, concurrent micro-batches and config 3's buckets "
                          "replay side by side on their own streams; 0 = one after the other"),
    "KRRN_PLAN_BUDGET_GB": ("48", "device memory the KRRN plan cache may hold before evicting the least "
                                  "recently used (B, S, N) plan"),
    "KRRN_DIAG_DROP": ("", "comma list of C-ABI entry points left out of new plans: a what-if timing "
                           "diagnostic (profiles/whatif.sh); outputs are meaningless with it set"),
    # --- kernel path selection (each alternative is a kept, tested path)
    "KRRN_WINO": ("1", "3x3 stride-1 convs on the Winograd kernels; 0 = the implicit-GEMM conv"),
    "KRRN_WINO_X3": ("1", "Winograd with split-bf16 MFMAs (f32 accuracy); 0 = the f32 Winograd"),
    "KRRN_WINO4": ("1", "the heads' wide 3x3 convs on the split-bf16 Winograd F(4x4, 3x3); 0 = F(2x2, 3x3)"),
    "KRRN_FUSE_EARLY": ("1", "HRNet fuse terms that read one branch start on that branch's stream before the join"),
    "KRRN_MODULE_STREAMS": ("1", "consecutive HRNet modules of a stage keep each branch on its stream (no barrier between them)"),
    "KRRN_STAGE_STREAMS": ("1", "with KRRN_MODULE_STREAMS, HRNet stages chain per branch stream too (transitions on their branch's stream)"),
    "KRRN_FUSION_EARLY": ("1", "the fusion work that reads only the input cloud runs beside the HRNet phase (side stream)"),
    "KRRN_FUSE_EDGES": ("1", "each HRNet fuse output waits for exactly its branches (capture edges); 0 = module barrier"),
    "KRRN_HEAD_FUSE": ("1", "a <= 4-output final 1x1 fused into the head's last split Winograd; 0 = two launches"),
    "KRRN_SMALL_CONV": ("1", "HRNet branch / fuse convs on the LDS-slab conv_small kernel; 0 = implicit GEMM"),
    "KRRN_GEMM_1X1": ("1", "stride-1 1x1 convs as plain GEMMs; 0 = implicit-GEMM conv"),
    "KRRN_CONVT_S2": ("1", "stride-2 transposed convs with 128 outputs on the all-classes-per-block kernel (convt.hip); 0 = the grouped implicit GEMM"),
    "KRRN_DECONV_FOLD": ("1", "fold last_layer_2 into the deconv (272 instead of 400 input channels); "
                              "0 = the literal cat + deconv"),
    "KRRN_FUSE_ID_FIRST": ("1", "HRNet fuse sums start from the identity branch; 0 = the reference's j order"),
    "KRRN_BLAS": ("1", "GEMMs no hand-written kernel takes go to hipBLASLt; 0 = the implicit-GEMM conv"),
    "KRRN_GEMM_X3": ("1", "GEMMs with K >= 256 on the split-bf16 GEMM"),
    "KRRN_GEMM_PANEL": ("1", "K = 64 / 128 GEMMs on the A-stationary panel GEMM"),
    "KRRN_SPLITK": ("1", "split-K for implicit-GEMM convs with few output tiles; 0 = never"),
    "KRRN_TBASE_EARLY": ("1", "TBase conv1's level-1 half runs as soon as level 1 is done (side stream)"),
    "KRRN_TBASE_GATHER": ("1", "TBase conv1 / conv2 by linearity on the fusion's level rows (gathered "
                               "GEMM); 0 = on the materialised 1280-wide concat"),
    "KRRN_POSE_AT": ("level1", "where the fused pose step forks off the forward plan: level1 / level2 / heads"),
    "KRRN_FUSION_CHUNK": ("16", "crops per chunk of the level-0 GCN GEMM + gather-conv, through a chunk-sized "
                                "Y buffer per branch (0 = the whole batch at once; same results)"),
}


def text(name: str) -> Optional[str]:
    if name not in KNOBS:
        raise KeyError(f"{name} is not a declared knob (pose_estimation_amd/knobs.py)")
    return os.environ.get(name, KNOBS[name][0])


def flag(name: str) -> bool:
    return text(name) == "1"


def integer(name: str) -> int:
    return int(text(name))
