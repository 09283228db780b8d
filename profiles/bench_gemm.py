"""Micro-bench: krrn_conv2d_f32 as a plain GEMM (the GCN `feature_map @ weights` and TBase shapes)
over the tile menu, vs hipBLASLt (torch.mm, f32). usage: python3 profiles/bench_gemm.py
env SHAPES="M,K,N[,a_cs];..." TILES="1,2,..." X3=1 """
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import ops  # noqa: E402
from pose_estimation_amd.runtime import TILE_SHAPES, Plan, add_conv, ptr  # noqa: E402

dev = torch.device("cuda", 0)
shapes = [(64000, 128, 1024, 384), (16000, 128, 1024, 384), (3968, 384, 4096, 384), (3968, 512, 4096, 512)]
if os.environ.get("SHAPES"):
    shapes = [tuple(int(v) for v in t.split(",")) for t in os.environ["SHAPES"].split(";")]
tiles = [int(t) for t in os.environ.get("TILES", ",".join(str(k) for k in TILE_SHAPES)).split(",")]
X3 = os.environ.get("X3") == "1"  # also krrn_conv2d_x3_f32 (split-bf16 operands) per tile


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


for shp in shapes:
    M, K, N = shp[:3]
    a_cs = shp[3] if len(shp) > 3 else K
    g = torch.Generator().manual_seed(0)
    A = torch.randn(M, a_cs, generator=g).to(dev)
    W = (0.05 * torch.randn(N, K, generator=g)).to(dev)
    scale = torch.ones(N, device=dev)
    bias = torch.zeros(N, device=dev)
    ref = A[:, :K] @ W.t()
    fl = 2.0 * M * N * K
    line = [f"M{M} K{K} N{N}:"]
    W3 = ops.conv_weights_x3(W)
    for t in tiles:
        for x3 in ((False, True) if X3 else (False,)):
            out = torch.zeros(M, N, device=dev)
            plan = Plan(dev)
            add_conv(plan, x=ptr(A), x_cs=a_cs, x_co=0, B=1, Hi=1, Wi=M, cin_p=K, Hg=1, Wg=M, in_s=1, taps=[(0, 0)],
                     wt=ptr(W), N=N, n_store=N, scale=ptr(scale), bias=ptr(bias), out=ptr(out), out_cs=N, out_co=0,
                     Ho=1, Wo=M, tile=t, splits=1, wt3=ptr(W3) if x3 else None)
            ms = ev_time(lambda: plan.run({}))
            err = float((out - ref).abs().max() / ref.abs().max())
            line.append(f"{'x3 ' if x3 else ''}t{t}{TILE_SHAPES[t]} {ms*1e3:.1f}us {fl/ms/1e9:.0f}TF"
                        + (" ERR" if err > 1e-5 else ""))
    from pose_estimation_amd import _lib
    from pose_estimation_amd.runtime import P
    st = P(torch.cuda.current_stream().cuda_stream)
    import ctypes
    h = ctypes.c_void_p()
    wsb = ctypes.c_longlong()
    _lib.check(_lib.lib().krrn_blas_gemm_create(M, N, K, a_cs, N, 1, 0, 0, 1, 0, 0, 0, 0, 64 << 20, ctypes.byref(h),
                                                ctypes.byref(wsb)), "blas create")
    ws = torch.empty(max(wsb.value, 16), dtype=torch.uint8, device=dev)
    out = torch.zeros(M, N, device=dev)
    fn = lambda: _lib.check(_lib.lib().krrn_blas_gemm_run(h, ptr(A), ptr(W), ptr(bias), ptr(None), ptr(out), ptr(ws),  # noqa: E731
                                                          wsb.value, st), "blas run")
    ms = ev_time(fn)
    o1 = out.clone()
    fn()
    torch.cuda.synchronize()
    err = float((out - ref).abs().max() / ref.abs().max())
    line.append(f"LT {ms*1e3:.1f}us {fl/ms/1e9:.0f}TF ws={wsb.value}" + (" ERR" if err > 1e-5 else "") +
                ("" if torch.equal(o1, out) else " NONDET"))
    _lib.lib().krrn_blas_gemm_destroy(h)
    w3f = ops.gemm_weights_x3(W)
    out = torch.zeros(M, N, device=dev)
    fn = lambda: _lib.check(_lib.lib().krrn_gemm_x3_f32(ptr(A), a_cs, M, K, N, ptr(w3f), ptr(bias), ptr(None), 0,  # noqa: E731
                                                        ptr(out), N, 0, 1, 0, 0, 0, st), "gemm_x3")
    if K % 32 == 0 and N % 128 == 0:
        ms = ev_time(fn)
        err = float((out - ref).abs().max() / ref.abs().max())
        line.append(f"GX3 {ms*1e3:.1f}us {fl/ms/1e9:.0f}TF" + (" ERR" if err > 1e-5 else ""))
    Ac = A[:, :K].contiguous()
    Wt = W.t().contiguous()
    ms = ev_time(lambda: torch.mm(Ac, Wt))
    line.append(f"torch.mm {ms*1e3:.1f}us {fl/ms/1e9:.0f}TF")
    print(" | ".join(line), flush=True)
