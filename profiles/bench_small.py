"""Micro-bench of krrn_conv_small_f32 on the HRNet-W18 branch BasicBlock convs at B = 64 (the
plan's (nw, ks) per shape, ops.small_conv_config): back-to-back launch throughput (us per launch
over 50 launches) and single-launch latency (median of 30 event-bracketed launches, synchronised
in between). KRRN_HIP_LIB selects a kernel-variant build (profiles/build_variant.sh); SWEEP=1 times
every (nw, ks) instead of the plan's.

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
    cfgs = [ops.small_conv_config(B * H * H, (cp + 15) // 16, cp)]
    if os.environ.get("SWEEP"):
        cfgs = [(nw, ks) for nw in (1, 2, 3) for ks in (1, 2, 4) if nw <= (cp + 15) // 16]
    for nw, ks in cfgs:
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
        # a dependent chain of 8 launches (input and output swapped each time) in one hipGraph: the
        # per-conv time of a branch's BasicBlock chain in the step's graph
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(gs):
            gst = P(gs.cuda_stream)
            with torch.cuda.graph(graph, stream=gs):
                for i in range(8):
                    src, dst = (x, out) if i % 2 == 0 else (out, x)
                    _lib.check(fn(ptr(src), cp, 0, B, H, H, cp, ptr(wp), cp, cp, ptr(sc), ptr(bi), ptr(res), cp, 0,
                                  ptr(dst), cp, 0, 1, 3, 1, nw, ks, gst), "small")
        torch.cuda.current_stream().wait_stream(gs)
        graph.replay()
        torch.cuda.synchronize()
        a.record()
        for _ in range(20):
            graph.replay()
        b.record()
        torch.cuda.synchronize()
        chain = a.elapsed_time(b) / 20 / 8 * 1e3
        x.copy_(torch.randn(B, H, H, cp, generator=g).to(dev))
        fl = 2.0 * B * H * H * cp * cp * 9
        print(f"{tag:18s} C{cp:3d} {H:2d}px nw {nw} ks {ks}: back-to-back {thr:6.1f} us  single {statistics.median(lat):6.1f} us"
              f"  graph chain {chain:6.1f} us  {fl / thr / 1e6:6.1f} TF/s", flush=True)
