"""Micro-bench: krrn_basic_block_x3_f32 (fused BasicBlock) against two krrn_conv_small_f32 launches
on the HRNet-W18 branch shapes at B = 64, back-to-back launch time, over the rows-per-block menu
(env TS = "0,2,4,8": 0 = ops.bb_tile_rows). KRRN_HIP_LIB selects a kernel-variant build.

usage (GPU box): python3 profiles/bench_bb.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 64))
TS = [int(t) for t in os.environ.get("TS", "0,1,2,4,8").split(",")]
L = _lib.lib()
st = P(torch.cuda.current_stream().cuda_stream)
tag = os.path.basename(os.environ.get("KRRN_HIP_LIB", "in-tree"))


def ev_time(fn, reps=40):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


SHAPES = [(20, 30), (36, 15), (72, 8), (144, 4)]
if os.environ.get("SHAPES_IDX"):  # e.g. "0" (PMC runs: keep the dispatch count small)
    SHAPES = [SHAPES[int(i)] for i in os.environ["SHAPES_IDX"].split(",")]
for C, H in SHAPES:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, H, H, C, generator=g).to(dev)
    w = [(torch.randn(C, 9 * C, generator=g) / (3 * C ** 0.5)).to(dev) for _ in range(2)]
    wb = [ops.bb_weights_x3(t, C) for t in w]
    sc = torch.ones(C, device=dev)
    bi = torch.zeros(C, device=dev)
    h = torch.zeros(B, H, H, C, device=dev)
    out = torch.zeros(B, H, H, C, device=dev)
    nw, ks = ops.small_conv_config(B * H * H, (C + 15) // 16, C)

    def two_small():
        _lib.check(L.krrn_conv_small_f32(ptr(x), C, 0, B, H, H, C, ptr(w[0]), C, C, ptr(sc), ptr(bi), P(0), 0, 0,
                                         ptr(h), C, 0, 1, 3, 1, nw, ks, st), "small")
        _lib.check(L.krrn_conv_small_f32(ptr(h), C, 0, B, H, H, C, ptr(w[1]), C, C, ptr(sc), ptr(bi), ptr(x), C, 0,
                                         ptr(out), C, 0, 1, 3, 1, nw, ks, st), "small")
    t2 = ev_time(two_small)
    ref = out.clone()
    line = [f"{tag:14s} C{C:3d} {H:2d}px: 2x small {t2:6.1f} us"]
    for T in TS:
        TT = T or ops.bb_tile_rows(B, H, H, C)
        if TT > H:
            continue

        def fused():
            _lib.check(L.krrn_basic_block_x3_f32(ptr(x), C, 0, B, H, H, C, ptr(wb[0]), ptr(sc), ptr(bi), ptr(wb[1]),
                                                 ptr(sc), ptr(bi), ptr(out), C, 0, TT, st), "bb")
        try:
            t = ev_time(fused)
        except RuntimeError:
            continue
        err = float((out - ref).abs().max())
        line.append(f"T{TT}{'*' if T == 0 else ''} {t:6.1f}" + (f" (err {err:.1e})" if err > 1e-3 else ""))
    print(" | ".join(line), flush=True)
