"""Micro-bench: krrn_conv3x3_wino_f32 vs MIOpen (torch conv2d) on the step's shapes."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.nn as nn
from pose_estimation_amd import ops, _lib
from pose_estimation_amd.runtime import P, ptr
dev = torch.device("cuda", 0)
shapes = [(64, 128, 128, 120, 120), (64, 128, 128, 60, 60), (64, 272, 272, 30, 30)]
if os.environ.get("SWEEP"): shapes = [(64, c, 128, 120, 120) for c in (32, 64, 128, 256)]
if os.environ.get("SHAPE"): shapes = [shapes[int(os.environ["SHAPE"])]]
if os.environ.get("SHAPES"):  # "B,cin,cout,H,W;..." e.g. the HRNet branch convs
    shapes = [tuple(int(v) for v in t.split(",")) for t in os.environ["SHAPES"].split(";")]
NOMIO = os.environ.get("NOMIO")
def ev_time(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
for B, cin, cout, H, W in shapes:
    g = torch.Generator().manual_seed(0)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
    with torch.no_grad(): conv.weight.copy_(0.05 * torch.randn(conv.weight.shape, generator=g))
    x = torch.randn(B, cin, H, W, generator=g).to(dev)
    xa = ops.new_act(B, H, W, cin, dev, cs=cin)
    xa.t.copy_(x.permute(0, 2, 3, 1))
    U = ops.wino_weights(conv, dev, cin_p=cin)
    out = ops.new_act(B, H, W, cout, dev, cs=cout)
    st = P(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    def run():
        _lib.check(L.krrn_conv3x3_wino_f32(ptr(xa.t), xa.cs, 0, B, H, W, cin, ptr(U), cout, cout, ptr(None), ptr(None),
                                           ptr(None), 0, 0, ptr(out.t), out.cs, 0, int(os.environ.get('RELU', '0')), st), "wino")
    ms = ev_time(run)
    cg = conv.to(dev)
    with torch.no_grad():
        ref = cg(x)
        mm = ev_time(lambda: cg(x)) if not NOMIO else 1.0
    err = float((out.t.permute(0, 3, 1, 2) - ref).abs().max() / ref.abs().max())
    fl = 2.0 * B * H * W * cin * cout * 9
    print(f"B{B} {cin}->{cout} {H}x{W}: wino {ms*1e3:8.1f} us {fl/ms/1e9:6.1f} TF(alg) {fl/2.25/ms/1e9:6.1f} TF(mfma) | miopen {mm*1e3:8.1f} us {fl/mm/1e9:6.1f} TF | rel err {err:.2e}", flush=True)
