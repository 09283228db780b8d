"""krrn_gemm_x3_f32 (split-bf16 GEMM, gemm_x3.hip) vs a plain PyTorch fp32 reference of the same op
(the GCN `feature_map @ weights` of gcn3d.py:125-127 / 184-186 and TBase's Conv1d chain): f32
tolerance against an f64 product, and within f32 rounding of torch's own f32 GEMM."""
import ctypes

import pytest
import torch

from pose_estimation_amd import _lib, ops
from pose_estimation_amd.runtime import P, ptr

pytestmark = pytest.mark.gpu


def _run(A, a_off, lda, M, K, N, W, bias, res, ldr, out, ldo, relu, batch=1, a_grp=0, o_grp=0, r_grp=0):
    w3 = ops.gemm_weights_x3(W)
    st = _lib.lib().krrn_gemm_x3_f32(P(A.data_ptr() + 4 * a_off), lda, M, K, N, ptr(w3), ptr(bias), ptr(res), ldr,
                                    ptr(out), ldo, int(relu), batch, a_grp, o_grp, r_grp,
                                    P(torch.cuda.current_stream().cuda_stream))
    _lib.check(st, "gemm_x3")
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,K,N,lda,a_off,relu,with_res", [
    (1000, 128, 256, 384, 128, True, False),   # GCN level-1 shape, channel slice of a 384-wide row
    (130, 384, 128, 384, 0, False, True),      # row tail, residual (TBase P1)
    (4000, 1024, 256, 1024, 0, True, False),   # TBase conv2
    (257, 256, 512, 260, 4, True, True)])
def test_gemm_x3_vs_torch(dev, M, K, N, lda, a_off, relu, with_res):
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn(M, lda + 4, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    bias = (0.1 * torch.randn(N, generator=g)).to(dev)
    res = torch.randn(M, N + 4, generator=g).to(dev) if with_res else None
    out = torch.full((M, N + 8), 7.0, device=dev)
    _run(A, a_off, lda + 4, M, K, N, W, bias, res, N + 4, out, N + 8, relu)
    Aw = A[:, a_off:a_off + K]
    ref64 = Aw.double() @ W.double().t() + bias.double()
    ref32 = Aw @ W.t() + bias
    if with_res:
        ref64 = ref64 + res[:, :N].double()
        ref32 = ref32 + res[:, :N]
    if relu:
        ref64, ref32 = ref64.clamp_min(0), ref32.clamp_min(0)
    got = out[:, :N]
    scale = float(ref64.abs().max())
    err = float((got.double() - ref64).abs().max())
    err32 = float((ref32.double() - ref64).abs().max())
    # f32 accuracy: the split kernel's error is of the order of torch's own f32 GEMM error
    assert err <= max(4 * err32, 2e-6 * scale), (err, err32, scale)
    assert torch.all(out[:, N:] == 7.0), "wrote past N"


def test_gemm_x3_batched(dev):
    """Strided groups (TBase's per-crop row subsets): group b reads A rows [b*a_grp, +M), writes
    out rows [b*o_grp, +M)."""
    g = torch.Generator().manual_seed(5)
    B, Nrows, M, K, N = 3, 300, 250, 384, 256
    A = torch.randn(B, Nrows, K, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    res = torch.randn(B, M, N, generator=g).to(dev)
    out = torch.zeros(B, M, N, device=dev)
    _run(A, 0, K, M, K, N, W, None, res, N, out, N, False, batch=B, a_grp=Nrows * K, o_grp=M * N, r_grp=M * N)
    ref = torch.einsum("bmk,nk->bmn", A[:, :M].double(), W.double()) + res.double()
    assert float((out.double() - ref).abs().max()) <= 2e-6 * float(ref.abs().max())


def test_gemm_x3_rejects(dev):
    A = torch.zeros(64, 128, device=dev)
    W = torch.zeros(128, 128, device=dev)
    out = torch.zeros(64, 128, device=dev)
    w3 = ops.gemm_weights_x3(W)
    L = _lib.lib()
    s = P(torch.cuda.current_stream().cuda_stream)
    assert L.krrn_gemm_x3_f32(ptr(A), 128, 64, 100, 128, ptr(w3), P(0), P(0), 0, ptr(out), 128, 0, 1, 0, 0, 0, s) < 0
    assert L.krrn_gemm_x3_f32(ptr(A), 128, 64, 128, 96, ptr(w3), P(0), P(0), 0, ptr(out), 128, 0, 1, 0, 0, 0, s) < 0
    assert L.krrn_gemm_x3_f32(P(A.data_ptr() + 4), 128, 64, 128, 128, ptr(w3), P(0), P(0), 0, ptr(out), 128, 0, 1, 0,
                              0, 0, s) < 0
    assert L.krrn_gemm_x3_f32(P(0), 128, 64, 128, 128, ptr(w3), P(0), P(0), 0, ptr(out), 128, 0, 1, 0, 0, 0, s) < 0


def _run_panel(A, a_off, lda, M, K, N, W, bias, res, ldr, out, ldo, relu, csplit=1):
    wp = ops.gemm_weights_panel(W)
    st = _lib.lib().krrn_gemm_panel_x3_f32(P(A.data_ptr() + 4 * a_off), lda, M, K, N, ptr(wp), ptr(bias), ptr(res),
                                          ldr, ptr(out), ldo, int(relu), csplit,
                                          P(torch.cuda.current_stream().cuda_stream))
    _lib.check(st, "gemm_panel_x3")
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,K,N,lda,a_off,relu,with_res,csplit", [
    (1000, 128, 1024, 384, 128, False, False, 1),  # GCN level-0/1 shape: a branch slice of the 384-wide rows
    (1000, 128, 1024, 384, 256, False, False, 4),  # column ranges (level 1 fills the chip this way)
    (77, 128, 96, 132, 4, True, False, 2),         # row tail (one partial panel), ReLU, ragged split
    (77, 64, 96, 132, 4, True, True, 2),           # the same with a residual (K = 64)
    (3000, 64, 256, 64, 0, True, True, 1)])        # layer1's 64 -> 256 1x1 (residual + ReLU)
def test_gemm_panel_vs_torch(dev, M, K, N, lda, a_off, relu, with_res, csplit):
    """krrn_gemm_panel_x3_f32 (A-stationary split-bf16 GEMM, gemm_panel.hip) vs torch f64 / f32."""
    g = torch.Generator().manual_seed(M + K + N + csplit)
    A = torch.randn(M, lda, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    bias = (0.1 * torch.randn(N, generator=g)).to(dev)
    res = torch.randn(M, N + 4, generator=g).to(dev) if with_res else None
    out = torch.full((M, N + 8), 7.0, device=dev)
    _run_panel(A, a_off, lda, M, K, N, W, bias, res, N + 4, out, N + 8, relu, csplit)
    Aw = A[:, a_off:a_off + K]
    ref64 = Aw.double() @ W.double().t() + bias.double()
    ref32 = Aw @ W.t() + bias
    if with_res:
        ref64 = ref64 + res[:, :N].double()
        ref32 = ref32 + res[:, :N]
    if relu:
        ref64, ref32 = ref64.clamp_min(0), ref32.clamp_min(0)
    got = out[:, :N]
    scale = float(ref64.abs().max())
    err = float((got.double() - ref64).abs().max())
    err32 = float((ref32.double() - ref64).abs().max())
    assert err <= max(4 * err32, 2e-6 * scale), (err, err32, scale)
    assert torch.all(out[:, N:] == 7.0), "wrote past N"


@pytest.mark.parametrize("M,K,N,ldo,ldr,out_off,with_res", [
    (77, 128, 96, 101, 0, 0, False),   # ldo % 4 != 0, row tail
    (77, 64, 96, 100, 99, 0, True),    # ldr % 4 != 0 with the residual, row tail
    (130, 64, 64, 68, 68, 1, True),    # out one float off 16-B alignment, residual, row tail
    (130, 128, 128, 132, 0, 3, False)])  # out three floats off, K = 128
def test_gemm_panel_scalar_epilogue(dev, M, K, N, ldo, ldr, out_off, with_res):
    """The g.vec == 0 epilogue of krrn_gemm_panel_x3_f32 (output / residual not float4-addressable:
    dword stores, scalar residual reads) vs torch f64, and nothing written outside the out view."""
    g = torch.Generator().manual_seed(M + K + N + ldo)
    A = torch.randn(M, K + 4, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    bias = (0.1 * torch.randn(N, generator=g)).to(dev)
    res = torch.randn(M * ldr + 8, generator=g).to(dev) if with_res else None
    buf = torch.full((out_off + M * ldo + 8,), 7.0, device=dev)
    wp = ops.gemm_weights_panel(W)
    st = _lib.lib().krrn_gemm_panel_x3_f32(ptr(A), K + 4, M, K, N, ptr(wp), ptr(bias), ptr(res), ldr,
                                          P(buf.data_ptr() + 4 * out_off), ldo, 1, 1,
                                          P(torch.cuda.current_stream().cuda_stream))
    _lib.check(st, "gemm_panel_x3 (scalar epilogue)")
    torch.cuda.synchronize()
    ref = A[:, :K].double() @ W.double().t() + bias.double()
    if with_res:
        ref = ref + res[:M * ldr].view(M, ldr)[:, :N].double()
    ref = ref.clamp_min(0)
    got = buf[out_off:out_off + M * ldo].view(M, ldo)
    err = float((got[:, :N].double() - ref).abs().max())
    assert err <= 2e-6 * float(ref.abs().max()), err
    assert torch.all(got[:, N:] == 7.0) and torch.all(buf[:out_off] == 7.0) and torch.all(buf[out_off + M * ldo:] == 7.0)


def test_gemm_panel_rejects(dev):
    A = torch.zeros(64, 128, device=dev)
    W = torch.zeros(128, 128, device=dev)
    out = torch.zeros(64, 128, device=dev)
    wp = ops.gemm_weights_panel(W)
    L = _lib.lib()
    s = P(torch.cuda.current_stream().cuda_stream)
    assert L.krrn_gemm_panel_x3_f32(ptr(A), 128, 64, 96, 128, ptr(wp), P(0), P(0), 0, ptr(out), 128, 0, 1, s) < 0
    assert L.krrn_gemm_panel_x3_f32(ptr(A), 128, 64, 128, 100, ptr(wp), P(0), P(0), 0, ptr(out), 128, 0, 1, s) < 0
    assert L.krrn_gemm_panel_x3_f32(P(A.data_ptr() + 4), 128, 64, 128, 128, ptr(wp), P(0), P(0), 0, ptr(out), 128, 0,
                                    1, s) < 0
    assert L.krrn_gemm_panel_x3_f32(P(0), 128, 64, 128, 128, ptr(wp), P(0), P(0), 0, ptr(out), 128, 0, 1, s) < 0
    # K = 128 with a residual: the 128-VGPR activation chain leaves no room for the residual tile: refused
    assert L.krrn_gemm_panel_x3_f32(ptr(A), 128, 64, 128, 128, ptr(wp), P(0), ptr(out), 128, ptr(out), 128, 0, 1,
                                    s) == -4


def test_gemm_x3_group_row_bias(dev):
    """ldr = 0: one res row per group, added to every row of the group (TBase's per-crop one-hot
    column + BN shift folded into conv1's level rows, posenet.emit_tbase_level1)."""
    g = torch.Generator().manual_seed(11)
    B, M, K, N = 4, 250, 384, 256
    A = torch.randn(B, M, K, generator=g).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    b2 = torch.randn(B, N, generator=g).to(dev)
    out = torch.zeros(B, M, N, device=dev)
    _run(A, 0, K, M, K, N, W, None, b2, 0, out, N, False, batch=B, a_grp=M * K, o_grp=M * N, r_grp=N)
    ref = torch.einsum("bmk,nk->bmn", A.double(), W.double()) + b2.double()[:, None, :]
    assert float((out.double() - ref).abs().max()) <= 2e-6 * float(ref.abs().max())


@pytest.mark.parametrize("B,npts,n1,n2", [(3, 300, 75, 18), (2, 1000, 250, 62), (1, 130, 40, 10)])
def test_gemm_x3_gather_vs_torch(dev, B, npts, n1, n2):
    """krrn_gemm_x3_gather_f32: TBase conv2 on h1 = ReLU(P1[b, ia] + P2[b, ib]) gathered while the
    operand is staged (posenet.py:51-96 by linearity) vs torch on the materialised h1."""
    g = torch.Generator().manual_seed(npts + n1)
    K, N = 1024, 256
    P1 = torch.randn(B, n1, K, generator=g).to(dev)
    P2 = torch.randn(B, n2, K, generator=g).to(dev)
    ia = torch.randint(0, n1, (B, npts), generator=g, dtype=torch.int32).to(dev)
    ib = torch.randint(0, n2, (B, npts), generator=g, dtype=torch.int32).to(dev)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    bias = (0.1 * torch.randn(N, generator=g)).to(dev)
    out = torch.full((B * npts, N + 4), 7.0, device=dev)
    w3 = ops.gemm_weights_x3(W)
    st = _lib.lib().krrn_gemm_x3_gather_f32(ptr(ia), ptr(P1), n1 * K, K, ptr(ib), ptr(P2), n2 * K, K, npts, B, K, N,
                                           ptr(w3), ptr(bias), ptr(out), N + 4, 1,
                                           P(torch.cuda.current_stream().cuda_stream))
    _lib.check(st, "gemm_x3_gather")
    torch.cuda.synchronize()
    bi = torch.arange(B, device=dev)[:, None]
    h1 = (P1[bi, ia.long()] + P2[bi, ib.long()]).clamp_min(0).reshape(B * npts, K)
    ref64 = (h1.double() @ W.double().t() + bias.double()).clamp_min(0)
    ref32 = (h1 @ W.t() + bias).clamp_min(0)
    err = float((out[:, :N].double() - ref64).abs().max())
    err32 = float((ref32.double() - ref64).abs().max())
    assert err <= max(4 * err32, 2e-6 * float(ref64.abs().max())), (err, err32)
    assert torch.all(out[:, N:] == 7.0), "wrote past N"
    # identical to the non-gathered kernel on the materialised h1 (same staging arithmetic)
    out2 = torch.zeros(B * npts, N, device=dev)
    _run(h1.contiguous(), 0, K, B * npts, K, N, W, bias, None, 0, out2, N, True)
    assert torch.equal(out[:, :N], out2)
