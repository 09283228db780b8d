"""Micro-bench: the four W18 stage-4 branch convs (18/36/72/144 channels at S/4 .. S/32, B = 64) as
four krrn_conv_small_f32 launches on one stream, on four streams, and as one
krrn_conv_small_group_f32 launch; each variant repeated `DEPTH` times back to back (a module's
block chain).

usage (GPU box): python3 profiles/bench_small_group.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, SmallDesc, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 64))
DEPTH = int(os.environ.get("DEPTH", 8))
L = _lib.lib()
shapes = [(20, 30), (36, 15), (72, 8), (144, 4)]
g = torch.Generator().manual_seed(0)
probs = []
for cp, H in shapes:
    nw, ks = ops.small_conv_config(B * H * H, (cp + 15) // 16, cp)
    x = torch.randn(B, H, H, cp, generator=g).to(dev)
    w = (0.05 * torch.randn(cp, 9 * cp, generator=g)).to(dev)
    out = torch.empty(B, H, H, cp, device=dev)
    probs.append(dict(x=x, w=w, out=out, cp=cp, H=H, nw=nw, ks=ks))
streams = [torch.cuda.Stream(dev) for _ in shapes]


def single(p, st):
    _lib.check(L.krrn_conv_small_f32(ptr(p["x"]), p["cp"], 0, B, p["H"], p["H"], p["cp"], ptr(p["w"]), p["cp"],
                                        p["cp"], P(0), P(0), P(0), 0, 0, ptr(p["out"]), p["cp"], 0, 1, 3, 1, p["nw"],
                                        p["ks"], P(st.cuda_stream)), "small")


arr = (SmallDesc * len(probs))(*[SmallDesc(in_=ptr(p["x"]), in_cs=p["cp"], in_co=0, B=B, H=p["H"], W=p["H"],
                                           cin=p["cp"], wt=ptr(p["w"]), N=p["cp"], n_store=p["cp"], scale=P(0),
                                           bias=P(0), res=P(0), res_cs=0, res_co=0, out=ptr(p["out"]),
                                           out_cs=p["cp"], out_co=0, relu=1, ksize=3, stride=1, nw=p["nw"], ks=p["ks"])
                                 for p in probs])


def run_serial():
    st = torch.cuda.current_stream()
    for _ in range(DEPTH):
        for p in probs:
            single(p, st)


def run_streams():
    main = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(main)
    for p, s in zip(probs, streams):
        for _ in range(DEPTH):
            single(p, s)
    for s in streams:
        main.wait_stream(s)


def run_group():
    st = torch.cuda.current_stream()
    for _ in range(DEPTH):
        _lib.check(L.krrn_conv_small_group_f32(ctypes.cast(arr, P), len(probs), P(st.cuda_stream)), "group")


def graph_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        gr.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for p in probs:
    t = graph_time(lambda: [single(p, torch.cuda.current_stream()) for _ in range(DEPTH)])
    print(f"C{p['cp']:3d} {p['H']:2d}x{p['H']:2d} <{p['nw']},{p['ks']}> alone: {t * 1e3 / DEPTH:6.1f} us/conv", flush=True)
for name, fn in (("serial", run_serial), ("4 streams", run_streams), ("group", run_group)):
    print(f"{name:10s}: {graph_time(fn) * 1e3 / DEPTH:6.1f} us per depth", flush=True)
