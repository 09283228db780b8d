"""Host-side weight packers (CPU): the layouts the HIP kernels index, checked element by element."""
import torch

from pose_estimation_amd import ops


def _bf16_to_f32(words: torch.Tensor, hi: bool) -> torch.Tensor:
    """The bf16 half (low or high 16 bits) of int32 words as f32."""
    w = words.to(torch.int64) & 0xFFFFFFFF
    bits = (w >> 16) if hi else (w & 0xFFFF)
    return (bits << 16).to(torch.int32).view(torch.float32)


def test_kchunk_weights_order():
    """krrn_conv_desc.k_chunk = q: k = ((c / q) * ntaps + tap) * q + c % q."""
    N, ntaps, cin, q = 8, 4, 32, 16
    w = torch.arange(N * ntaps * cin, dtype=torch.float32).reshape(N, ntaps * cin)
    r = ops.kchunk_weights(w, ntaps, cin, q)
    for n in (0, 5):
        for tap in range(ntaps):
            for c in range(cin):
                k_new = ((c // q) * ntaps + tap) * q + c % q
                assert r[n, k_new] == w[n, tap * cin + c]


def test_panel_chain_layout_reconstructs_weights():
    """ops.gemm_weights_panel: word (nb, g, lane, i) of the [m h] plane and (nb, g, lane, j) of
    the [l] plane hold the split terms of W[32 nb + lane % 32, 8 g + 4 (lane / 32) + e], and
    h + m + l == W exactly."""
    g = torch.Generator().manual_seed(0)
    N, K = 64, 32
    W = torch.randn(N, K, generator=g)
    P = ops.gemm_weights_panel(W)
    assert P.shape == (N // 32, K // 8, 384) and P.dtype == torch.int32
    mh = P[..., :256].reshape(N // 32, K // 8, 64, 4)
    lp = P[..., 256:].reshape(N // 32, K // 8, 64, 2)
    for nb in range(N // 32):
        for gi in range(K // 8):
            for lane in (0, 7, 31, 32, 45, 63):
                n, k0 = 32 * nb + lane % 32, 8 * gi + 4 * (lane // 32)
                words_m, words_h, words_l = mh[nb, gi, lane, :2], mh[nb, gi, lane, 2:], lp[nb, gi, lane]
                for e in range(4):
                    m = _bf16_to_f32(words_m[e // 2], e % 2 == 1)
                    h = _bf16_to_f32(words_h[e // 2], e % 2 == 1)
                    l_ = _bf16_to_f32(words_l[e // 2], e % 2 == 1)
                    # three exact bf16 terms: the f32 sum is exact in f64
                    assert float(h.double() + m.double() + l_.double()) == float(W[n, k0 + e])

