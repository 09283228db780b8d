"""krrn_resize_bilinear_f32 (HRNet fuse / final upsample, myhrnet.py:242-245, 511-516; the heads'
UpsamplingBilinear2d, krrn.py:56, 78) against torch's F.interpolate in f32, both conventions,
with the fused residual add + ReLU, on NHWC channel slices; upsampling (2x2 outputs per thread,
odd output sizes) and downsampling (one output per thread)."""
import pytest
import torch
import torch.nn.functional as F

from pose_estimation_amd import _lib
from pose_estimation_amd.runtime import P, ptr


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,Hi,Wi,Ho,Wo,align,fused", [
    # >= 2^21 output quads: the 2x2-outputs-per-thread upsampling kernel (the heads' upsample, an odd size)
    (24, 128, 60, 60, 120, 120, True, False), (24, 128, 61, 45, 121, 90, False, True),
    # one output per thread: small upsamples, downsampling, a 1-pixel source
    (3, 128, 60, 60, 120, 120, True, False), (3, 20, 15, 15, 30, 30, False, True), (3, 36, 8, 8, 15, 15, False, True),
    (3, 144, 4, 4, 30, 30, False, False), (3, 1024, 5, 7, 9, 13, True, True), (3, 8, 3, 5, 40, 11, False, False),
    (3, 16, 30, 30, 15, 15, False, False), (3, 12, 9, 7, 4, 5, True, True), (3, 4, 1, 1, 3, 2, True, False)])
def test_resize_matches_torch(dev, B, C, Hi, Wi, Ho, Wo, align, fused):
    g = torch.Generator().manual_seed(C + Ho)
    pad = 4
    x = torch.randn(B, C, Hi, Wi, generator=g)
    ref = F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=align)
    base = torch.randn(B, C, Ho, Wo, generator=g)
    if fused:
        ref = torch.relu(ref + base)
    xin = torch.zeros(B, Hi, Wi, C + 2 * pad)
    xin[..., pad:pad + C] = x.permute(0, 2, 3, 1)
    out = torch.zeros(B, Ho, Wo, C + pad)
    out[..., pad:] = base.permute(0, 2, 3, 1)
    xd, od = xin.to(dev), out.to(dev)
    add = od if fused else None
    _lib.call("krrn_resize_bilinear_f32", ptr(xd), B, Hi, Wi, C + 2 * pad, pad, C, ptr(od), Ho, Wo, C + pad, pad,
              ptr(add), C + pad, pad, int(align), int(fused), P(torch.cuda.current_stream().cuda_stream))
    got = od.cpu()[..., pad:].permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
