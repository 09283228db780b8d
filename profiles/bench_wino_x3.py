"""Micro-bench: krrn_conv3x3_wino_f32 (f32 MFMA), krrn_conv3x3_wino_x3_f32 (split-bf16 F(2x2,3x3))
and krrn_conv3x3_wino4_x3_f32 (split-bf16 F(4x4,3x3)) on the step's Winograd shapes: time per launch,
and the error of each against an f64 CPU conv of the first 2 images (max |err| / max |ref| and RMS
err / RMS ref).

usage (GPU box): python3 profiles/bench_wino_x3.py      (KERNELS=x3,w4 selects; REPS=n)
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

dev = torch.device("cuda", 0)
shapes = [(64, 128, 128, 120, 120), (64, 128, 128, 60, 60), (64, 272, 272, 30, 30), (64, 64, 64, 60, 60)]
if os.environ.get("SHAPES"):
    shapes = [tuple(int(v) for v in t.split(",")) for t in os.environ["SHAPES"].split(";")]
L = _lib.lib()


def ev_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for B, cin, cout, H, W in shapes:
    g = torch.Generator().manual_seed(0)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / (3.0 * cin ** 0.5))
    x = torch.relu(torch.randn(B, cin, H, W, generator=g))
    xa = ops.new_act(B, H, W, cin, dev, cs=cin)
    xa.t.copy_(x.permute(0, 2, 3, 1).to(dev))
    U = ops.wino_weights(conv, dev, cin_p=cin)
    U3 = ops.wino_weights_x3(U)
    U4 = ops.wino_weights_x3(ops.wino4_weights(conv, dev, cin_p=cin)) if cin % 8 == 0 else None
    out = ops.new_act(B, H, W, cout, dev, cs=cout)
    st = P(torch.cuda.current_stream().cuda_stream)
    with torch.no_grad():
        ref = (torch.nn.functional.conv2d(x[:2].double(), conv.weight.double(), padding=1).permute(0, 2, 3, 1)
               if not os.environ.get("NOREF") else None)

    def f32():
        _lib.check(L.krrn_conv3x3_wino_f32(ptr(xa.t), xa.cs, 0, B, H, W, cin, ptr(U), cout, cout, ptr(None), ptr(None),
                                           ptr(None), 0, 0, ptr(out.t), out.cs, 0, 0, st), "wino")

    def x3():
        _lib.check(L.krrn_conv3x3_wino_x3_f32(ptr(xa.t), xa.cs, 0, B, H, W, cin, ptr(U3), cout, cout, ptr(None),
                                              ptr(None), ptr(None), 0, 0, ptr(out.t), out.cs, 0, 0, st), "wino_x3")

    def w4():
        _lib.check(L.krrn_conv3x3_wino4_x3_f32(ptr(xa.t), xa.cs, 0, B, H, W, cin, ptr(U4), cout, cout, ptr(None),
                                               ptr(None), ptr(None), 0, 0, ptr(out.t), out.cs, 0, 0, st), "wino4_x3")

    fl = 2.0 * B * H * W * cin * cout * 9
    line = f"B{B} {cin}->{cout} {H}x{W}:"
    kinds = os.environ.get("KERNELS", "f32,x3,w4").split(",")
    for name, fn in (("f32", f32), ("x3", x3), ("w4", w4)):
        if name not in kinds or (name == "w4" and U4 is None):
            continue
        out.t.zero_()
        ms = ev_time(fn, int(os.environ.get("REPS", "10")))
        line += f" | {name} {ms * 1e3:7.1f} us {fl / ms / 1e9:6.1f} TF(alg)"
        if ref is not None:
            e = out.t[:2, :, :, :cout].double().cpu() - ref
            line += f" max {float(e.abs().max() / ref.abs().max()):.2e} rms {float(e.norm() / ref.norm()):.2e}"
    print(line, flush=True)
