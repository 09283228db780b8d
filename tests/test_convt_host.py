"""Host side of krrn_convT_s2_x3_f32 (CPU): ops.convT_weights_x3's split weight planes and class/tap
table, checked by decoding them and evaluating the kernel's sub-pixel sum in f64 against
torch's ConvTranspose2d (the formula convt.hip implements; the GPU test runs the kernel itself)."""
import pytest
import torch
import torch.nn as nn

from pose_estimation_amd import ops


def _decode(U3: torch.Tensor, nck: int, N: int) -> torch.Tensor:
    """wino_weights_x3 planes -> f32 [nck][16][N][8] (h + m + l)."""
    n = nck * 16 * N * 2
    mh = U3[:n * 8].view(nck, 16, N, 2, 8).float()
    lo = U3[n * 8:].view(nck, 16, N, 2, 4).float()
    u = mh[..., :4] + mh[..., 4:] + lo  # m + h + l per channel
    return u.reshape(nck, 16, N, 8)


@pytest.mark.parametrize("cin,k,op", [(24, 4, 0), (16, 3, 1), (8, 2, 0)])
def test_convT_weights_and_table(cin, k, op):
    g = torch.Generator().manual_seed(cin + k)
    B, H, W, N = 2, 5, 7, 128
    convT = nn.ConvTranspose2d(cin, N, k, 2, 1, output_padding=op, bias=False)
    with torch.no_grad():
        convT.weight.copy_(torch.randn(convT.weight.shape, generator=g))
    spec = ops.make_convT(convT, None, "cpu")
    U3, table = ops.convT_weights_x3(spec)
    nck = spec.cin_p // 8
    U = _decode(U3, nck, N).double()  # [nck][class * 4 + tap][N][8]
    # the three bf16 terms reproduce the f32 weights exactly
    for c, taps in enumerate(spec.taps):
        w = spec.wt[c].double().reshape(N, len(taps), nck, 8)
        for t in range(len(taps)):
            assert torch.equal(U[:, 4 * c + t], w[:, t].permute(1, 0, 2))
        for t in range(len(taps), 4):
            assert not U[:, 4 * c + t].any()
    # the table: tap count, then (dy + 1) * 3 + (dx + 1)
    assert [table[5 * c] for c in range(4)] == [len(t) for t in spec.taps]
    for c, taps in enumerate(spec.taps):
        for t, (dy, dx) in enumerate(taps):
            assert table[5 * c + 1 + t] == (dy + 1) * 3 + (dx + 1)
    # the kernel's sum, from the decoded planes and the table, in f64
    x = torch.randn(B, cin, H, W, generator=g, dtype=torch.float64)
    ref = torch.nn.functional.conv_transpose2d(x, convT.weight.double(), stride=2, padding=1, output_padding=op)
    Ho, Wo = ref.shape[2:]
    xp = torch.zeros(B, 8 * nck, H + 2, W + 2, dtype=torch.float64)
    xp[:, :cin, 1:H + 1, 1:W + 1] = x
    Wk = U.permute(1, 2, 0, 3).reshape(16, N, 8 * nck)  # [class * 4 + tap][n][k]
    got = torch.zeros_like(ref)
    for c in range(4):
        py, px = c >> 1, c & 1
        acc = torch.zeros(B, N, H, W, dtype=torch.float64)
        for t in range(table[5 * c]):
            code = table[5 * c + 1 + t]
            dy, dx = code // 3 - 1, code % 3 - 1
            patch = xp[:, :, 1 + dy:1 + dy + H, 1 + dx:1 + dx + W]  # in[a + dy][b + dx]
            acc += torch.einsum("bkhw,nk->bnhw", patch, Wk[4 * c + t])
        oh, ow = (Ho - py + 1) // 2, (Wo - px + 1) // 2
        got[:, :, py::2, px::2] = acc[:, :, :oh, :ow]
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)


def test_convT_s2_eligible():
    g = torch.Generator().manual_seed(1)

    def act(c, cs, co=0, H=30, W=30):
        return ops.Act(torch.empty(0), 1, H, W, cs, co, c)

    for k, op, cin, cout, ok in ((4, 0, 272, 128, True), (3, 1, 128, 128, True), (4, 0, 272, 64, False),
                                 (5, 0, 64, 128, False), (3, 1, 12, 128, False)):
        convT = nn.ConvTranspose2d(cin, cout, k, 2, 1 if k < 5 else 2, output_padding=op, bias=False)
        spec = ops.make_convT(convT, None, "cpu")
        x = act(cin, ops.pad4(cin))
        out = act(cout, ops.pad4(cout), H=60, W=60)
        assert ops.convT_s2_eligible(spec, x, out, None) == ok, (k, op, cin, cout)
        if ok:
            assert not ops.convT_s2_eligible(spec, x, out, out)  # a residual is not supported
