"""Micro-bench: the F(4x4) head form (krrn_conv3x3_wino4_x3_head_f32: NMLNet's last 120-px conv +
nml_final, p1 = 3) against the plain launch of the same conv (krrn_conv3x3_wino4_x3_f32), B = 64,
128 -> 128, 120 x 120: time per launch, alternating REPS-launch bursts.

usage (GPU box): python3 profiles/bench_wino_head.py   (REPS=n, ROUNDS=n; KRRN_HIP_LIB=... for an A/B)
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B, C, H, W, p1 = 64, 128, 120, 120, 3
REPS, ROUNDS = int(os.environ.get("REPS", 200)), int(os.environ.get("ROUNDS", 3))
L = _lib.lib()
g = torch.Generator().manual_seed(0)
conv = nn.Conv2d(C, C, 3, 1, 1, bias=False)
with torch.no_grad():
    conv.weight.copy_(0.05 * torch.randn(conv.weight.shape, generator=g))
spec = ops.make_conv(conv, None, dev, cin_p=C)
U3 = ops.wino_weights_x3(ops.wino4_weights(conv, dev, cin_p=C))
xa = ops.new_act(B, H, W, C, dev)
xa.t.copy_(torch.randn(xa.t.shape, generator=g).to(dev))
w1 = (0.1 * torch.randn(4, C, generator=g)).to(dev)
b1 = torch.zeros(4, device=dev)
part = torch.empty(2 * B * H * W * 4, device=dev)
out = torch.empty(B, p1, H, W, device=dev)
full = ops.new_act(B, H, W, C, dev)
st = P(torch.cuda.current_stream().cuda_stream)


def head():
    _lib.check(L.krrn_conv3x3_wino4_x3_head_f32(ptr(xa.t), xa.cs, 0, B, H, W, C, ptr(U3), C, ptr(spec.scale),
                                                 ptr(spec.bias), ptr(None), 0, 0, 1, ptr(w1), ptr(b1), p1, ptr(part),
                                                 ptr(out), p1, st), "head")


def plain():
    _lib.check(L.krrn_conv3x3_wino4_x3_f32(ptr(xa.t), xa.cs, 0, B, H, W, C, ptr(U3), C, C, ptr(spec.scale),
                                            ptr(spec.bias), ptr(None), 0, 0, ptr(full.t), full.cs, 0, 1, st), "plain")


def ev_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for r in range(ROUNDS):
    print(f"round {r}: head {ev_time(head, REPS):7.1f} us (2 launches: conv + finish) | plain {ev_time(plain, REPS):7.1f} us",
          flush=True)
