"""Where the F(4x4) Winograd kernel's time goes, from per-wave cycle stamps (timing study only).

Needs a build with -DKRRN_W4_TRACE=1 (profiles/build_variant.sh NAME winograd4 "-DKRRN_W4_TRACE=1"),
selected with KRRN_HIP_LIB. One 120-px launch (B=64, 128 -> 128); the first 256 blocks (one per CU)
record, per wave: kernel start, prologue end, per chunk (16) its start / after component 4 / the end of
its component loop (then the barrier), the epilogue start and end. Prints per-phase cycle means
(over blocks, per wave index) and the chunk loop's split into M/T work and barrier wait.

usage (GPU box): KRRN_HIP_LIB=build/exp/tr.so python3 profiles/w4_trace.py [B H cin]
"""
import ctypes
import os
import sys

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B, H, cin = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 120, 128)
W, cout = H, 128
L = _lib.lib()
T = ctypes.CDLL(os.environ["KRRN_HIP_LIB"])
g = torch.Generator().manual_seed(0)
conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
with torch.no_grad():
    conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / (3.0 * cin ** 0.5))
xa = ops.new_act(B, H, W, cin, dev, cs=cin)
xa.t.copy_(torch.relu(torch.randn(B, H, W, cin, generator=g)).to(dev))
U4 = ops.wino_weights_x3(ops.wino4_weights(conv, dev, cin_p=cin))
out = ops.new_act(B, H, W, cout, dev, cs=cout)
st = P(torch.cuda.current_stream().cuda_stream)


def run():
    _lib.check(L.krrn_conv3x3_wino4_x3_f32(ptr(xa.t), xa.cs, 0, B, H, W, cin, ptr(U4), cout, cout, ptr(None),
                                           ptr(None), ptr(None), 0, 0, ptr(out.t), out.cs, 0, 0, st), "wino4")


for _ in range(3):
    run()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
run()
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) * 1e3
KT = 52
buf = np.zeros(256 * 8 * KT, dtype=np.uint32)
assert T.krrn_w4_trace_copy(buf.ctypes.data_as(ctypes.c_void_p)) == 0
tr = buf.reshape(256, 8, KT).astype(np.int64)
nck = min(16, cin // 8)


def d(i, j):  # cycles from stamp i to stamp j (u32 wrap)
    return (tr[:, :, j] - tr[:, :, i]) % (1 << 32)


k0 = tr[:, :, 48]
span = (tr[:, :, 51] - k0.min(axis=1, keepdims=True)) % (1 << 32)
print(f"B{B} {cin}->{cout} {H}x{W}: launch {us:.1f} us; first-wave block span {span.max(axis=1).mean():.0f} cyc")
rows = {"prologue": d(48, 49), "chunk0 wait->start": d(49, 0)}
m1 = np.stack([d(3 * c, 3 * c + 1) for c in range(nck)], -1)
m2 = np.stack([d(3 * c + 1, 3 * c + 2) for c in range(nck)], -1)
bar = np.stack([d(3 * c + 2, 3 * c + 3) for c in range(nck - 1)], -1)
rows["chunk k0-4 (mean)"] = m1.mean(-1)
rows["chunk k5-8 (mean)"] = m2.mean(-1)
rows["chunk barrier (mean)"] = bar.mean(-1)
rows["last chunk end -> epilogue"] = d(3 * (nck - 1) + 2, 50)
rows["epilogue"] = d(50, 51)
print(f"{'phase':30s} " + " ".join(f"w{w:<6d}" for w in range(8)) + "  mean")
for name, v in rows.items():
    per_w = v.mean(axis=0)
    print(f"{name:30s} " + " ".join(f"{x:7.0f}" for x in per_w) + f"  {v.mean():7.0f}")
tot = (m1 + m2).sum(-1) + bar.sum(-1)
print(f"chunk loop total {tot.mean():.0f} cyc: M/T work {(m1 + m2).sum(-1).mean():.0f}, barrier {bar.sum(-1).mean():.0f}")
print("per-chunk k0-4 / k5-8 / barrier, wave-mean:")
for c in range(nck):
    print(f"  ck{c:2d} {m1[:, :, c].mean():6.0f} {m2[:, :, c].mean():6.0f} "
          f"{bar[:, :, c].mean() if c < nck - 1 else 0:6.0f}")
