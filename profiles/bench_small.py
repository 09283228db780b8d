"""Micro-bench of krrn_conv_small_f32 on the HRNet-W18 branch BasicBlock convs at B = 64 (the
plan's (nw, ks) per shape, ops.small_conv_config): back-to-back launch throughput (us per launch
over 50 launches) and single-launch latency (median of 30 event-bracketed launches, synchronised
in between). KRRN_HIP_LIB selects a kernel-variant build (profiles/build_variant.sh).

usage (GPU box): python3 profiles/bench_small.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 64))
shapes = [(20, 30), (36, 15), (72, 8), (144, 4)]  # (padded C, side)
L = _lib.lib()
st = P(torch.cuda.current_stream().cuda_stream)
tag = os.path.basename(os.environ.get("KRRN_HIP_LIB", "in-tree"))
for cp, H in shapes:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, H, H, cp, generator=g).to(dev)
    w = (0.05 * torch.randn(cp, 9 * cp, generator=g)).to(dev)
    res = torch.randn(B, H, H, cp, generator=g).to(dev)
    sc = torch.ones(cp, device=dev)
    bi = torch.zeros(cp, device=dev)
    out = torch.zeros(B, H, H, cp, device=dev)
    nw, ks = ops.small_conv_config(B * H * H, (cp + 15) // 16, cp)

    fn, wp = L.krrn_conv_small_f32, w

    def run():
        _lib.check(fn(ptr(x), cp, 0, B, H, H, cp, ptr(wp), cp, cp, ptr(sc), ptr(bi), ptr(res), cp, 0,
                      ptr(out), cp, 0, 1, 3, 1, nw, ks, st), "small")
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        run()
    b.record()
    torch.cuda.synchronize()
    thr = a.elapsed_time(b) / 50 * 1e3
    lat = []
    for _ in range(30):
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        lat.append(a.elapsed_time(b) * 1e3)
    fl = 2.0 * B * H * H * cp * cp * 9
    print(f"{tag:18s} C{cp:3d} {H:2d}px nw {nw} ks {ks}: back-to-back {thr:6.1f} us  single {statistics.median(lat):6.1f} us"
          f"  {fl / thr / 1e6:6.1f} TF/s", flush=True)
