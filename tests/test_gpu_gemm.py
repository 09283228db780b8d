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
    (77, 128, 96, 132, 4, True, True, 2),          # row tail (one partial panel), residual, ReLU, ragged split
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
