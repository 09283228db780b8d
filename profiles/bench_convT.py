"""Micro-bench: the step's two transposed convs (HRNet deconv 4x4 272 -> 128 and XYZNet 3x3
128 -> 128, both 30 -> 60 px, B = 64) as one grouped split-bf16 launch per tile shape, built the
way hrnet.emit_conv builds them (parity classes, channel-chunk k order).

usage (GPU box): python3 profiles/bench_convT.py   (TILES=1,6,8 the grouped tiles, TILES= none; "s2" = the
all-classes-per-block kernel, krrn_convT_s2_x3_f32; CASE=0 / 1 one of the two convs, e.g. for a
per-conv rocprofv3 --pmc pass)
"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import ops  # noqa: E402
from pose_estimation_amd.runtime import Plan, add_conv_group, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", 64))
cases = [("convT4 272->128 30->60", nn.ConvTranspose2d(272, 128, 4, 2, 1, bias=False)),
         ("convT3 128->128 30->60", nn.ConvTranspose2d(128, 128, 3, 2, 1, output_padding=1, bias=False))]


def build(spec, xa, out, tile, q):
    plan = Plan(dev)
    np_ = ops.pad4(spec.cout)
    probs = []
    for cls, (taps, (ooy, oox)) in enumerate(zip(spec.taps, spec.cls_off)):
        w = ops.kchunk_weights(spec.wt[cls], len(taps), spec.cin_p, q) if q else spec.wt[cls]
        w3 = ops.conv_weights_x3(w)
        plan.buffers.append(w3)
        probs.append(dict(x=ptr(xa.t), x_cs=xa.cs, x_co=xa.co, B=xa.B, Hi=xa.H, Wi=xa.W, cin_p=spec.cin_p, Hg=xa.H,
                          Wg=xa.W, in_s=1, taps=taps, wt=ptr(w3), N=np_, n_store=np_, scale=ptr(spec.scale),
                          bias=ptr(spec.bias), res=None, res_cs=0, res_co=0, out=ptr(out.t), out_cs=out.cs,
                          out_co=out.co, Ho=out.H, Wo=out.W, osy=2, osx=2, ooy=ooy, oox=oox, relu=True,
                          cin=spec.cin, cout=spec.cout, k_chunk=q))
    add_conv_group(plan, probs, tile=tile, tag="bench", x3=True)
    return plan


def ev_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


if os.environ.get("CASE"):
    cases = [cases[int(os.environ["CASE"])]]
for name, conv in cases:
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        conv.weight.copy_(0.05 * torch.randn(conv.weight.shape, generator=g))
    spec = ops.make_convT(conv, None, dev)
    xa = ops.new_act(B, 30, 30, conv.in_channels, dev)
    xa.t.copy_(torch.randn(xa.t.shape, generator=g).to(dev))
    out = ops.new_act(B, 60, 60, spec.cout, dev)
    line, ref = name + ":", None
    for tile in [int(t) for t in os.environ.get("TILES", "1,6,8").split(",") if t]:
        for q in (0, 16):
            try:
                plan = build(spec, xa, out, tile, q)
                ms = ev_time(lambda: plan.run({}))
            except RuntimeError as e:
                line += f" | t{tile} q{q} n/a ({str(e).split(': ')[-1][:24]})"
                continue
            got = out.t.clone()
            ref = got if ref is None else ref
            err = float((got - ref).abs().max() / ref.abs().max())
            line += f" | t{tile} q{q} {ms * 1e3:6.1f} us ({err:.1e})"
    U3, table = ops.convT_weights_x3(spec)
    from pose_estimation_amd import _lib  # noqa: E402
    from pose_estimation_amd.runtime import P  # noqa: E402

    def s2():
        _lib.check(_lib.lib().krrn_convT_s2_x3_f32(ptr(xa.t), xa.cs, xa.co, B, 30, 30, spec.cin_p, table, ptr(U3), 128,
                                                   ptr(spec.scale), ptr(spec.bias), 1, ptr(out.t), out.cs, out.co,
                                                   60, 60, P(torch.cuda.current_stream().cuda_stream)), "convT_s2")
    ms = ev_time(s2)
    got = out.t.clone()
    err = float((got - ref).abs().max() / ref.abs().max()) if ref is not None else float("nan")
    line += f" | s2 {ms * 1e3:6.1f} us ({err:.1e})"
    print(line, flush=True)
