"""krrn_basic_block_x3_f32 (conv_bb.hip: one HRNet BasicBlock per launch, lib/network/hrnet/myhrnet.py:34-63)
vs a plain PyTorch reference of the same block: f32 tolerance against torch f32, f32-level error
against an f64 evaluation, pad channels kept zero, nothing written outside the output slice."""
import pytest
import torch
import torch.nn as nn

from pose_estimation_amd import _lib, ops
from pose_estimation_amd.runtime import P, ptr

pytestmark = pytest.mark.gpu


def _bn(c, g):
    bn = nn.BatchNorm2d(c).eval()
    with torch.no_grad():
        bn.weight.copy_(1 + 0.1 * torch.randn(c, generator=g))
        bn.bias.copy_(0.1 * torch.randn(c, generator=g))
        bn.running_mean.copy_(0.1 * torch.randn(c, generator=g))
        bn.running_var.copy_(0.5 + torch.rand(c, generator=g))
    return bn


def _block(c, g):
    convs = [nn.Conv2d(c, c, 3, 1, 1, bias=False) for _ in range(2)]
    with torch.no_grad():
        for cv in convs:
            cv.weight.copy_(torch.randn(cv.weight.shape, generator=g) / (3 * c ** 0.5))
    return convs[0], _bn(c, g), convs[1], _bn(c, g)


def _ref(x, c1, b1, c2, b2):
    return torch.relu(b2(c2(torch.relu(b1(c1(x))))) + x)


@pytest.mark.parametrize("c,H,T,co", [
    (18, 30, 0, 0), (18, 30, 3, 4), (18, 30, 1, 0),    # branch 0 (18 -> 20 physical channels)
    (36, 15, 0, 0), (36, 15, 1, 0),                    # branch 1
    (72, 8, 0, 8), (72, 8, 8, 0),                      # branch 2 (channel-split waves)
    (144, 4, 0, 0), (144, 4, 1, 0),                    # branch 3
    (32, 10, 0, 0)])                                   # W32-style width, whole channel tiles
def test_basic_block_vs_torch(dev, c, H, T, co):
    B = 3
    g = torch.Generator().manual_seed(c * 31 + H + T)
    c1, b1, c2, b2 = _block(c, g)
    x = torch.randn(B, c, H, H, generator=g)
    with torch.no_grad():
        ref32 = _ref(x, c1, b1, c2, b2)
        ref64 = _ref(x.double(), c1.double(), b1.double(), c2.double(), b2.double())
    C = ops.pad4(c)
    cs = C + co + 4
    xa = torch.zeros(B, H, H, cs)
    xa[..., co:co + c] = x.permute(0, 2, 3, 1)
    xa = xa.to(dev)
    s1 = ops.make_conv(c1.float(), b1.float(), dev, cin_p=C)
    s2 = ops.make_conv(c2.float(), b2.float(), dev, cin_p=C)
    w1, w2 = ops.bb_weights_x3(s1.wt[0], C), ops.bb_weights_x3(s2.wt[0], C)
    ocs, oco = C + 8, 4
    out = torch.full((B, H, H, ocs), float("nan"), device=dev)
    T = T or ops.bb_tile_rows(B, H, H, C)
    _lib.check(_lib.lib().krrn_basic_block_x3_f32(ptr(xa), cs, co, B, H, H, C, ptr(w1), ptr(s1.scale), ptr(s1.bias),
                                                  ptr(w2), ptr(s2.scale), ptr(s2.bias), ptr(out), ocs, oco, T,
                                                  P(torch.cuda.current_stream().cuda_stream)), "basic block")
    torch.cuda.synchronize()
    got = out[..., oco:oco + c].permute(0, 3, 1, 2).cpu()
    torch.testing.assert_close(got, ref32, rtol=2e-4, atol=2e-4)
    err = float((got.double() - ref64).abs().max())
    err32 = float((ref32.double() - ref64).abs().max())
    assert err <= max(4 * err32, 2e-6 * float(ref64.abs().max())), (err, err32)
    assert torch.count_nonzero(out[..., oco + c:oco + C]).item() == 0, "pad channels not zero"
    assert torch.isnan(out[..., :oco]).all() and torch.isnan(out[..., oco + C:]).all(), "wrote outside the slice"


def test_basic_block_rejects(dev):
    L = _lib.lib()
    s = P(torch.cuda.current_stream().cuda_stream)
    x = torch.zeros(1, 8, 8, 20, device=dev)
    w = torch.zeros(4096, dtype=torch.int32, device=dev)
    v = torch.zeros(20, device=dev)
    # aliasing in / out (the residual is re-read), misaligned channel offset, too much LDS
    assert L.krrn_basic_block_x3_f32(ptr(x), 20, 0, 1, 8, 8, 20, ptr(w), ptr(v), ptr(v), ptr(w), ptr(v), ptr(v), ptr(x),
                                     20, 0, 4, s) != 0
    assert L.krrn_basic_block_x3_f32(ptr(x), 20, 2, 1, 8, 8, 16, ptr(w), ptr(v), ptr(v), ptr(w), ptr(v), ptr(v),
                                     ptr(torch.zeros_like(x)), 20, 0, 4, s) != 0
    big = torch.zeros(1, 64, 64, 256, device=dev)
    assert L.krrn_basic_block_x3_f32(ptr(big), 256, 0, 1, 64, 64, 256, ptr(w), ptr(v), ptr(v), ptr(w), ptr(v), ptr(v),
                                     ptr(torch.zeros_like(big)), 256, 0, 64, s) != 0
