"""Micro-bench: krrn_conv2d_f32 against krrn_conv2d_x3_f32 (split-bf16 operands) per tile on the
step's implicit-GEMM shapes (the transposed convs' parity classes and a stride-2 conv), B = 64.

usage (GPU box): python3 profiles/bench_conv_x3.py
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 64))
cases = [("convT4 272->128 30->60", nn.ConvTranspose2d(272, 128, 4, 2, 1, bias=False), 30),
         ("convT3 128->128 60->120", nn.ConvTranspose2d(128, 128, 3, 2, 1, output_padding=1, bias=False), 60),
         ("conv3s2 64->64 120->60", nn.Conv2d(64, 64, 3, 2, 1, bias=False), 120)]


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


for name, conv, H in cases:
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        conv.weight.copy_(0.05 * torch.randn(conv.weight.shape, generator=g))
    cin = conv.in_channels
    spec = ops.make_conv(conv, None, dev) if isinstance(conv, nn.Conv2d) else ops.make_convT(conv, None, dev)
    xa = ops.new_act(B, H, H, cin, dev)
    xa.t.copy_(torch.randn(xa.t.shape, generator=g).to(dev))
    Ho, Wo = ops.conv_out_hw(spec, H, H)
    out = ops.new_act(B, Ho, Wo, spec.cout, dev)
    line = name + ":"
    for x3, tile in ((False, 8), (True, 8), (True, 7), (True, 1), (True, 4), (True, 2)):
        ms = ev_time(lambda: ops.conv2d(xa, spec, out, tile=tile, x3=x3))
        line += f" | {'x3' if x3 else 'f32'} t{tile} {ms * 1e3:7.1f} us"
    print(line, flush=True)
