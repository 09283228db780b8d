"""Micro-bench: krrn_conv2d_f32 on the HRNet-W18 branch BasicBlock convs (3x3, stride 1, C -> C at
B = 64) over the tile / split-K menu, against MIOpen (torch conv2d) on the same shape.

usage (GPU box): python3 profiles/bench_branch_conv.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib  # noqa: E402
from pose_estimation_amd.runtime import P, ptr, _iarr  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 64))
shapes = [(20, 18, 30), (36, 36, 15), (72, 72, 8), (144, 144, 4)]  # (padded C, logical C, side)
if os.environ.get("SHAPES_IDX"):  # e.g. "0,3" (PMC runs: keep the dispatch count small)
    shapes = [shapes[int(i)] for i in os.environ["SHAPES_IDX"].split(",")]
TILES = [int(t) for t in os.environ.get("TILES", "6,8,3,5").split(",")]
SPLITS = [int(t) for t in os.environ.get("SPLITS", "1,2,4,8").split(",")]
TAPS = [(dy, dx) for dy in (-1, 0, 1) for dx in (-1, 0, 1)]


def ev_time(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


L = _lib.lib()
st = P(torch.cuda.current_stream().cuda_stream)
for cp, c, H in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, H, H, cp, generator=g)
    x[..., c:] = 0
    w = 0.05 * torch.randn(cp, 9, cp, generator=g)  # [N][tap][cin]
    w[:, :, c:] = 0
    w[c:] = 0
    ref = F.conv2d(x.permute(0, 3, 1, 2), w.view(cp, 3, 3, cp).permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    xd, wd = x.to(dev), w.reshape(cp, 9 * cp).contiguous().to(dev)
    out = torch.zeros(B, H, H, cp, device=dev)
    ws = torch.empty(16 * B * H * H * cp, device=dev)
    fl = 2.0 * B * H * H * c * c * 9
    for tile in TILES:
        for splits in SPLITS:
            def run():
                _lib.check(L.krrn_conv2d_f32(ptr(xd), cp, 0, B, H, H, cp, H, H, 1, 9, _iarr([t[0] for t in TAPS]),
                                             _iarr([t[1] for t in TAPS]), ptr(wd), cp, cp, P(0), P(0), P(0), 1, P(0),
                                             0, 0, ptr(out), cp, 0, H, H, 1, 1, 0, 0, 0, 0, tile, splits, ptr(ws), st),
                           "conv")
            ms = ev_time(run)
            err = float((out.cpu() - ref).abs().max())
            print(f"C{c:3d} {H:2d}x{H:2d} tile {tile} splits {splits}: {ms*1e3:7.1f} us {fl/ms/1e9:6.1f} TF err {err:.1e}",
                  flush=True)
    for nw in [int(v) for v in os.environ.get("SMALL_NW", "1,2,3").split(",") if v]:
        for ks in [int(v) for v in os.environ.get("SMALL_KS", "1,2,4").split(",") if v]:
            def run_small():
                _lib.check(L.krrn_conv_small_f32(ptr(xd), cp, 0, B, H, H, cp, ptr(wd), cp, cp, P(0), P(0), P(0), 0,
                                                    0, ptr(out), cp, 0, 0, 3, 1, nw, ks, st), "small conv")
            ms = ev_time(run_small)
            err = float((out.cpu() - ref).abs().max())
            print(f"C{c:3d} {H:2d}x{H:2d} small nw {nw} ks {ks}: {ms*1e3:7.1f} us {fl/ms/1e9:6.1f} TF err {err:.1e}",
                  flush=True)
    xc = x.permute(0, 3, 1, 2)[:, :c].contiguous().to(dev)
    wc = w.view(cp, 3, 3, cp).permute(0, 3, 1, 2)[:c, :c].contiguous().to(dev)
    mm = ev_time(lambda: F.conv2d(xc, wc, padding=1)) if not os.environ.get("NOMIO") else float("nan")
    print(f"C{c:3d} {H:2d}x{H:2d} MIOpen NCHW: {mm*1e3:7.1f} us {fl/mm/1e9:6.1f} TF", flush=True)
