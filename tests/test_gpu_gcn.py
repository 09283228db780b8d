"""krrn_gcn_conv_f32 (Conv_layer, gcn3d.py:136-216) against a plain torch fp32 statement of the
same op. Neighbour lists: "local" ones (every neighbour within +-16 of the point's own index, as
pixel-ordered `choose` rows give) and fully random ones (the sampled levels), ragged n (not a
multiple of the block's 8 points), k = 10 / 7 / 16 (compile-time and runtime k paths).
"""
import pytest
import torch

from pose_estimation_amd import _lib
from pose_estimation_amd.runtime import P, ptr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _torch_conv_layer(idx, v, dn, Y, S, C, bn_s, bn_b, relu):
    B, n, k = idx.shape
    bi = torch.arange(B)[:, None, None]
    d = v[bi, idx.long()] - v[:, :, None, :]                              # [B, n, k, 3]
    d = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    theta = torch.relu(d @ dn)                                            # [B, n, k, S*C]
    sup = Y[bi, idx.long(), C:]                                           # [B, n, k, S*C]
    act = (theta * sup).max(dim=2).values.view(B, n, S, C).sum(dim=2)
    out = Y[:, :, :C] + act
    out = out * bn_s + bn_b
    return torch.relu(out) if relu else out


def _idx(B, n, k, mode, g):
    if mode == "local":
        w = 16
        off = torch.randint(-w, w + 1, (B, n, k), generator=g)
        base = torch.arange(n)[None, :, None]
        i = (base + off).clamp(0, n - 1)
        i = torch.where(i == base, (base + 1) % n, i)
    else:
        i = torch.randint(0, n, (B, n, k), generator=g)
    return i.to(torch.int32)


@pytest.mark.parametrize("B,n,k,mode", [(4, 1000, 10, "local"), (3, 250, 10, "local"), (2, 1000, 10, "random"),
                                        (2, 77, 7, "local"), (2, 300, 16, "local"), (1, 31, 10, "random")])
def test_gcn_conv_layer(dev, B, n, k, mode):
    S, C = 7, 128
    g = torch.Generator().manual_seed(n * 31 + k)
    idx = _idx(B, n, k, mode, g)
    v = torch.randn(B, n, 9, generator=g)                                 # fusion's [x y z nx ny nz r g b] rows
    dn = torch.randn(3, S * C, generator=g)
    dn = dn / dn.norm(dim=0, keepdim=True)
    Y = torch.randn(B, n, (S + 1) * C, generator=g)
    bn_s = 1 + 0.1 * torch.randn(C, generator=g)
    bn_b = 0.1 * torch.randn(C, generator=g)
    ref = _torch_conv_layer(idx, v[..., :3], dn, Y, S, C, bn_s, bn_b, True)
    L = _lib.lib()
    st = P(torch.cuda.current_stream().cuda_stream)
    d_idx, d_v, d_dn, d_Y = idx.to(dev), v.to(dev), dn.contiguous().to(dev), Y.to(dev)
    d_s, d_b = bn_s.to(dev), bn_b.to(dev)
    out = torch.full((B, n, C), float("nan"), device=dev)
    _lib.check(L.krrn_gcn_conv_f32(ptr(d_idx), n, k, ptr(d_v), n * 9, 9, 3, ptr(d_dn), S, C, ptr(d_Y), ptr(d_s),
                                   ptr(d_b), 1, ptr(out), n * C, C, B, st), "gcn conv")
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("B,n,k,has_y", [(4, 1000, 10, False), (2, 250, 8, True), (2, 77, 8, False),
                                         (3, 64, 10, True)])
def test_gcn_conv_surface_and_k8(dev, B, n, k, has_y):
    """Conv_surface (gcn3d.py:88-112: no Y, ReLU(max_k theta) summed over supports, no BN) and the
    k = 8 level-1 form of the test shapes, through the LDS-staged 3-D kernel."""
    S, C = 7, 128
    g = torch.Generator().manual_seed(n * 17 + k + int(has_y))
    idx = _idx(B, n, k, "local", g)
    v = torch.randn(B, n, 9, generator=g)
    dn = torch.randn(3, S * C, generator=g)
    dn = dn / dn.norm(dim=0, keepdim=True)
    bi = torch.arange(B)[:, None, None]
    if has_y:
        Y = torch.randn(B, n, (S + 1) * C, generator=g)
        ref = _torch_conv_layer(idx, v[..., :3], dn, Y, S, C, torch.ones(C), torch.zeros(C), False)
    else:
        Y = None
        d = v[bi, idx.long(), :3] - v[:, :, None, :3]
        d = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        ref = torch.relu((d @ dn).max(dim=2).values).view(B, n, S, C).sum(dim=2)
    L = _lib.lib()
    st = P(torch.cuda.current_stream().cuda_stream)
    d_idx, d_v, d_dn = idx.to(dev), v.to(dev), dn.contiguous().to(dev)
    d_Y = Y.to(dev) if has_y else None
    out = torch.full((B, n, C), float("nan"), device=dev)
    _lib.check(L.krrn_gcn_conv_f32(ptr(d_idx), n, k, ptr(d_v), n * 9, 9, 3, ptr(d_dn), S, C, ptr(d_Y), P(0), P(0), 0,
                                   ptr(out), n * C, C, B, st), "gcn conv")
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=2e-5)
