"""Thin Python wrappers over the C-ABI entry points of libkrrn_hip.so.

Tensors are used only as device-memory handles: every wrapper passes raw
``data_ptr()`` values, sizes and the current HIP stream to the library. No
arithmetic happens here.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib, knobs


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _int_array(vals: Sequence[int], n: int = 9):
    arr = (ctypes.c_int * n)()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def pad4(c: int) -> int:
    return (c + 3) // 4 * 4


@dataclass
class Act:
    """An NHWC activation: channels [co, co + cp) of a [B, H, W, cs] f32 buffer.

    ``c`` is the logical channel count (reference layout); ``cp = pad4(c)`` is the
    physical width the kernels read/write (pad channels are kept at exactly 0).
    """
    t: torch.Tensor
    B: int
    H: int
    W: int
    cs: int
    co: int
    c: int

    @property
    def cp(self) -> int:
        return pad4(self.c)

    def slice(self, co: int, c: int) -> "Act":
        return Act(self.t, self.B, self.H, self.W, self.cs, self.co + co, c)


def new_act(B: int, H: int, W: int, c: int, device, cs: Optional[int] = None) -> Act:
    cs = pad4(c) if cs is None else cs
    t = torch.zeros((B, H, W, cs), dtype=torch.float32, device=device)
    return Act(t, B, H, W, cs, 0, c)


@dataclass
class ConvSpec:
    """A folded convolution ready for krrn_conv2d_f32.

    ``wt``: [classes][Np, ntaps*cin_p]; ``taps``/``grid`` describe each launch class.
    For a plain conv there is one class; a stride-2 transposed conv has four
    (output parity classes, sub-pixel decomposition).
    """
    wt: List[torch.Tensor]
    taps: List[List[Tuple[int, int]]]
    cls_off: List[Tuple[int, int]]  # output offset (ooy, oox) per class
    scale: torch.Tensor
    bias: torch.Tensor
    cin_p: int
    cout: int
    stride: int      # input stride for normal convs
    kind: str        # "conv" | "convT"
    ksize: int
    pad: int
    cin: int = 0     # logical input channels (algorithmic FLOP count)


def conv_out_hw(spec: ConvSpec, H: int, W: int) -> Tuple[int, int]:
    if spec.kind == "conv":
        Ho = (H + 2 * spec.pad - spec.ksize) // spec.stride + 1
        Wo = (W + 2 * spec.pad - spec.ksize) // spec.stride + 1
        return Ho, Wo
    return 2 * H, 2 * W


def conv2d(x: Act, spec: ConvSpec, out: Act, res: Optional[Act] = None, relu: bool = False,
           bias2: Optional[torch.Tensor] = None, b2_div: int = 1, tile: int = 0, splits: int = 1,
           ws: Optional[torch.Tensor] = None, x3: bool = False):
    """out = act(BN(conv(x)) [+ bias2] [+ res]) written into ``out``'s channel slice; x3: on the
    bf16 matrix cores with split operands (krrn_conv2d_x3_f32, tiles 6 / 7 / 8)."""
    assert x.cp == spec.cin_p, (x.c, x.cp, spec.cin_p)
    Ho, Wo = out.H, out.W
    np_ = pad4(spec.cout)
    for cls, (taps, (ooy, oox)) in enumerate(zip(spec.taps, spec.cls_off)):
        if spec.kind == "conv":
            Hg, Wg, in_s, osy, osx = Ho, Wo, spec.stride, 1, 1
        else:
            Hg, Wg, in_s, osy, osx = x.H, x.W, 1, 2, 2
        dy = _int_array([t[0] for t in taps])
        dx = _int_array([t[1] for t in taps])
        if x3:
            from .runtime import conv_tile
            t = tile or conv_tile(x.B * Hg * Wg, np_, spec.cin_p * len(taps))
            if not hasattr(spec, "wt3"):
                spec.wt3 = [conv_weights_x3(w) for w in spec.wt]
            w3 = spec.wt3[cls]
            _lib.call("krrn_conv2d_x3_f32",
                      _ptr(x.t), x.cs, x.co, x.B, x.H, x.W, spec.cin_p, Hg, Wg, in_s, len(taps), dy, dx,
                      _ptr(w3), np_, np_, _ptr(spec.scale), _ptr(spec.bias), _ptr(bias2), b2_div,
                      _ptr(res.t if res is not None else None), res.cs if res is not None else 0,
                      res.co if res is not None else 0,
                      _ptr(out.t), out.cs, out.co, Ho, Wo, osy, osx, ooy, oox, int(relu), t, splits,
                      _ptr(ws), _stream())
            continue
        _lib.call("krrn_conv2d_f32",
                  _ptr(x.t), x.cs, x.co, x.B, x.H, x.W, spec.cin_p,
                  Hg, Wg, in_s, len(taps), dy, dx,
                  _ptr(spec.wt[cls]), np_, np_, _ptr(spec.scale), _ptr(spec.bias),
                  _ptr(bias2), b2_div,
                  _ptr(res.t if res is not None else None), res.cs if res is not None else 0,
                  res.co if res is not None else 0,
                  _ptr(out.t), out.cs, out.co, Ho, Wo, osy, osx, ooy, oox, int(relu), 0, tile, splits,
                  _ptr(ws), _stream())


def conv2d_nchw(x: Act, spec: ConvSpec, out: torch.Tensor, n_store: int, relu: bool = False, tile: int = 0):
    """Final 1x1 conv writing an NCHW [B, n_store, H, W] tensor (heads, krrn.py:97-98)."""
    assert spec.kind == "conv" and len(spec.taps) == 1
    B, C, Ho, Wo = out.shape
    np_ = pad4(spec.cout)
    taps = spec.taps[0]
    if not tile:
        from .runtime import conv_tile
        tile = conv_tile(B * Ho * Wo, np_, spec.cin_p, nchw=True)
    _lib.call("krrn_conv2d_f32",
              _ptr(x.t), x.cs, x.co, x.B, x.H, x.W, spec.cin_p,
              Ho, Wo, spec.stride, len(taps), _int_array([t[0] for t in taps]), _int_array([t[1] for t in taps]),
              _ptr(spec.wt[0]), np_, n_store, _ptr(spec.scale), _ptr(spec.bias), _ptr(None), 1,
              _ptr(None), 0, 0, _ptr(out), C, 0, Ho, Wo, 1, 1, 0, 0, int(relu), 1, tile, 1, _ptr(None), _stream())


def gemm(a: torch.Tensor, a_cs: int, a_co: int, M: int, spec: ConvSpec, out: torch.Tensor, out_cs: int,
         out_co: int, relu: bool = False, bias2: Optional[torch.Tensor] = None, b2_div: int = 1, tile: int = 0,
         splits: int = 1, ws: Optional[torch.Tensor] = None):
    """Row-major GEMM out[M, :N] = act(scale * (A[M, K] @ W^T) + bias [+ bias2]) via the conv kernel."""
    np_ = pad4(spec.cout)
    _lib.call("krrn_conv2d_f32",
              _ptr(a), a_cs, a_co, 1, 1, M, spec.cin_p, 1, M, 1, 1, _int_array([0]), _int_array([0]),
              _ptr(spec.wt[0]), np_, np_, _ptr(spec.scale), _ptr(spec.bias), _ptr(bias2), b2_div,
              _ptr(None), 0, 0, _ptr(out), out_cs, out_co, 1, M, 1, 1, 0, 0, int(relu), 0, tile, splits, _ptr(ws),
              _stream())


# ----------------------------------------------------------------------------------------
# Weight folding / packing (run once at plan build time; not on the per-step path)
# ----------------------------------------------------------------------------------------

def fold_bn(cout: int, conv_bias: Optional[torch.Tensor], bn: Optional[torch.nn.Module], device):
    """Eval-mode BN folded to (scale, bias): y = scale * conv + bias (BN eps from the module)."""
    np_ = pad4(cout)
    scale = torch.zeros(np_, dtype=torch.float64)
    bias = torch.zeros(np_, dtype=torch.float64)
    cb = conv_bias.detach().double().cpu() if conv_bias is not None else torch.zeros(cout, dtype=torch.float64)
    if bn is None:
        scale[:cout] = 1.0
        bias[:cout] = cb
    else:
        g = bn.weight.detach().double().cpu()
        b = bn.bias.detach().double().cpu()
        mu = bn.running_mean.detach().double().cpu()
        var = bn.running_var.detach().double().cpu()
        s = g / torch.sqrt(var + bn.eps)
        scale[:cout] = s
        bias[:cout] = (cb - mu) * s + b
    return scale.float().to(device), bias.float().to(device)


def _pack_taps(w: torch.Tensor, taps_k: List[Tuple[int, int]], cin_map: List[int], cin_p: int, cout: int):
    """w: [cout, cin, kh, kw] (conv layout) -> [pad4(cout), ntaps * cin_p], channel-mapped.

    cin_map[c] = physical channel of logical input channel c.
    """
    np_ = pad4(cout)
    nt = len(taps_k)
    out = torch.zeros(np_, nt, cin_p, dtype=torch.float32)
    idx = torch.tensor(cin_map, dtype=torch.long)
    for t, (ky, kx) in enumerate(taps_k):
        out[:cout, t, idx] = w[:, :, ky, kx].float()
    return out.reshape(np_, nt * cin_p).contiguous()


def make_conv(conv: torch.nn.Conv2d, bn: Optional[torch.nn.Module], device, cin_map: Optional[List[int]] = None,
              cin_p: Optional[int] = None) -> ConvSpec:
    w = conv.weight.detach().cpu()
    cout, cin, kh, kw = w.shape
    assert kh == kw
    k, s = kh, conv.stride[0]
    p = conv.padding
    if isinstance(p, str):  # 'same' (stride 1, odd kernel)
        pad = (k - 1) // 2
    else:
        pad = p[0]
    if cin_map is None:
        cin_map = list(range(cin))
    cin_p = pad4(max(cin_map) + 1) if cin_p is None else cin_p
    taps_k = [(ky, kx) for ky in range(k) for kx in range(k)]
    wt = _pack_taps(w, taps_k, cin_map, cin_p, cout).to(device)
    scale, bias = fold_bn(cout, conv.bias, bn, device)
    taps = [(ky - pad, kx - pad) for (ky, kx) in taps_k]
    return ConvSpec([wt], [taps], [(0, 0)], scale, bias, cin_p, cout, s, "conv", k, pad, len(cin_map))


# Winograd switches, read at import like every other knob (knobs.py)
WINO = knobs.flag("KRRN_WINO")
WINO4 = knobs.flag("KRRN_WINO4")

# Winograd F(2x2, 3x3) weight transform G (Lavin & Gray 2016): U = G g G^T
WINO_G = torch.tensor([[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]], dtype=torch.float64)


def wino_weights(conv: torch.nn.Conv2d, device, cin_map: Optional[List[int]] = None,
                 cin_p: Optional[int] = None) -> torch.Tensor:
    """[cout, cin, 3, 3] -> U f32 in the kernel's chunk-major order [ceil(cin_p/8)][16][pad4(cout)][8]
    (xi = 4u + v; channels past cin_p are zero), transformed in f64."""
    w = conv.weight.detach().cpu().double()
    cout, cin = w.shape[:2]
    if cin_map is None:
        cin_map = list(range(cin))
    cin_p = pad4(max(cin_map) + 1) if cin_p is None else cin_p
    u = torch.einsum("ui,ncij,vj->uvnc", WINO_G, w, WINO_G)  # [4, 4, cout, cin]
    out = torch.zeros(16, pad4(cout), cin_p, dtype=torch.float64)
    out[:, :cout, torch.tensor(cin_map, dtype=torch.long)] = u.reshape(16, cout, cin)
    nck = (cin_p + 7) // 8
    out = torch.nn.functional.pad(out, (0, 8 * nck - cin_p))
    out = out.view(16, pad4(cout), nck, 8).permute(2, 0, 1, 3)  # [chunk][xi][n][8]
    return out.float().contiguous().to(device)


# Winograd F(4x4, 3x3) weight transform G, points (0, +-1, +-2) (Lavin & Gray 2016): U = G g G^T
WINO4_G = torch.tensor([[1 / 4, 0.0, 0.0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6],
                        [1 / 24, 1 / 12, 1 / 6], [1 / 24, -1 / 12, 1 / 6], [0.0, 0.0, 1.0]], dtype=torch.float64)


def wino4_weights(conv: torch.nn.Conv2d, device, cin_map: Optional[List[int]] = None,
                  cin_p: Optional[int] = None) -> torch.Tensor:
    """[cout, cin, 3, 3] -> U f32 for krrn_conv3x3_wino4_x3_f32 in chunk-major order
    [ceil(cin_p/8)][36][pad4(cout)][8] (xi = 6u + v; channels past cin_p are zero), transformed in
    f64 (G's 1/6 and 1/24 are not exact in f32; the f32 rounding of U happens once, here)."""
    w = conv.weight.detach().cpu().double()
    cout, cin = w.shape[:2]
    if cin_map is None:
        cin_map = list(range(cin))
    cin_p = pad4(max(cin_map) + 1) if cin_p is None else cin_p
    u = torch.einsum("ui,ncij,vj->uvnc", WINO4_G, w, WINO4_G)  # [6, 6, cout, cin]
    out = torch.zeros(36, pad4(cout), cin_p, dtype=torch.float64)
    out[:, :cout, torch.tensor(cin_map, dtype=torch.long)] = u.reshape(36, cout, cin)
    nck = (cin_p + 7) // 8
    out = torch.nn.functional.pad(out, (0, 8 * nck - cin_p))
    out = out.view(36, pad4(cout), nck, 8).permute(2, 0, 1, 3)  # [chunk][xi][n][8]
    return out.float().contiguous().to(device)


def split_bf16x3(u: torch.Tensor):
    """f32 -> three bf16 terms, each the round-to-nearest of what the previous ones left:
    u = h + m + l exactly (24 significand bits), |m| <= 2^-8 |u|, |l| <= 2^-16 |u|."""
    u = u.float()
    h = u.bfloat16()
    r = u - h.float()
    m = r.bfloat16()
    l = (r - m.float()).bfloat16()
    return h, m, l


def wino_weights_x3(U: torch.Tensor) -> torch.Tensor:
    """wino_weights' U [nck][16][N][8] (or wino4_weights' [nck][36][N][8]) f32 -> the split planes
    krrn_conv3x3_wino_x3_f32 (krrn_conv3x3_wino4_x3_f32) reads, as one bf16 tensor:
    U_mh [nck][xi][N][half][m0..m3 h0..h3] then U_l [nck][xi][N][half][l0..l3]
    (half = channels 4 half .. 4 half + 3 of the chunk)."""
    h, m, l = split_bf16x3(U)
    nck, nxi, N, _ = U.shape
    h, m, l = (t.reshape(nck, nxi, N, 2, 4) for t in (h, m, l))
    mh = torch.cat([m, h], dim=-1).reshape(-1)
    return torch.cat([mh, l.reshape(-1)]).contiguous()


def convT_s2_eligible(spec: "ConvSpec", x, out, res) -> bool:
    """krrn_convT_s2_x3_f32 runs a stride-2 transposed conv with 128 outputs, taps within one input
    pixel of the grid point (padding 1, kernel <= 4), >= 8 input channels in whole chunks of 8, a
    16-byte aligned NHWC input and no residual: the backbone's deconv and XYZNet's first layer."""
    return (spec.kind == "convT" and len(spec.taps) == 4 and pad4(spec.cout) == 128 and res is None
            and all(1 <= len(t) <= 4 and all(-1 <= dy <= 1 and -1 <= dx <= 1 for dy, dx in t) for t in spec.taps)
            and spec.cin_p % 8 == 0 and x.cs % 4 == 0 and x.co % 4 == 0 and x.co + spec.cin_p <= x.cs
            and out.co + 128 <= out.cs and out.H <= 2 * x.H and out.W <= 2 * x.W
            and [tuple(o) for o in spec.cls_off] == [(0, 0), (0, 1), (1, 0), (1, 1)])


def convT_weights_x3(spec: "ConvSpec") -> Tuple[torch.Tensor, "ctypes.Array"]:
    """make_convT's per-class weights [N][taps * cin_p] -> (U3, cls_taps) for krrn_convT_s2_x3_f32:
    U [cin_p / 8][class * 4 + tap][N][8] f32 (zero for a class's missing taps) split into the
    wino_weights_x3 planes, and the 4 x 5 int table [tap count, (dy + 1) * 3 + (dx + 1) ...]."""
    N, cin_p = spec.wt[0].shape[0], spec.cin_p
    if spec.kind != "convT" or cin_p % 8 or len(spec.taps) != 4 or any(len(t) > 4 for t in spec.taps):
        raise ValueError("convT_weights_x3: a stride-2 transposed conv with cin_p % 8 == 0 and <= 4 taps per class")
    nck = cin_p // 8
    U = torch.zeros(nck, 16, N, 8, device=spec.wt[0].device)
    table = (ctypes.c_int * 20)()
    for c, taps in enumerate(spec.taps):
        w = spec.wt[c].float().reshape(N, len(taps), nck, 8)
        table[5 * c] = len(taps)
        for t, (dy, dx) in enumerate(taps):
            U[:, 4 * c + t] = w[:, t].permute(1, 0, 2)
            table[5 * c + 1 + t] = (dy + 1) * 3 + (dx + 1)
    return wino_weights_x3(U), table


def conv_weights_x3(wt: torch.Tensor) -> torch.Tensor:
    """krrn_conv2d_f32 weights [N][K] f32 -> the split chains krrn_conv2d_x3_f32 reads: bf16
    [N][K / 4][16], per 4 k the terms m0..m3 h0..h3 l0..l3 then 4 zeros (K a multiple of 4)."""
    N, K = wt.shape
    h, m, l = split_bf16x3(wt)
    h, m, l = (t.reshape(N, K // 4, 4) for t in (h, m, l))
    return torch.cat([m, h, l, torch.zeros_like(l)], dim=-1).contiguous()


def kchunk_weights(wt: torch.Tensor, ntaps: int, cin: int, q: int) -> torch.Tensor:
    """Conv weights [N][ntaps * cin] (k = tap * cin + c) -> the channel-chunk-major order of
    krrn_conv_desc.k_chunk = q: k = ((c / q) * ntaps + tap) * q + c % q."""
    N = wt.shape[0]
    return wt.reshape(N, ntaps, cin // q, q).permute(0, 2, 1, 3).reshape(N, ntaps * cin).contiguous()


def gemm_weights_x3(wt: torch.Tensor) -> torch.Tensor:
    """GEMM weights [N][K] f32 (scale folded) -> the wave fragments krrn_gemm_x3_f32 reads: int32
    [N/32][K/8][2][64][4]. Fragment (column block nb, 8-k group g, quad q) is one coalesced 1-KB
    wave load: lane fh*32 + nl holds, for column 32 nb + nl and k = 8 g + 4 fh .. + 3, the MFMA
    operand quad q of the split terms: q = 0 [h0..h3 l0..l3] (pairs with the activations' [h h]),
    q = 1 [m0..m3 h0..h3] (pairs with [h m] and [m l]). N % 32 == 0, K % 8 == 0."""
    N, K = wt.shape
    h, m, l = (t.reshape(N, K // 4, 4) for t in split_bf16x3(wt))
    c = torch.cat([h, l, m, h], dim=-1).contiguous()  # [N][K/4][16] bf16 = P0 | P1
    c = c.view(torch.int32).reshape(N // 32, 32, K // 8, 2, 2, 4)  # nb nl g fh q 4
    return c.permute(0, 2, 4, 3, 1, 5).contiguous()                 # nb g q fh nl 4


def quad_weights_x3(wt: torch.Tensor, N: int, K: int, kq_mult: int = 4) -> torch.Tensor:
    """Conv weights [>= N][>= K] f32 (k = tap * cin + c, ops.make_conv's packing) -> the split planes
    the channel-quad kernels read (krrn_conv1x1_nchw_x3_f32), int32: the
    [m h] plane [N16][KQp][4] (per output channel and channel quad kq: m0..m3 h0..h3 bf16) then the
    [l] plane [N16][KQp][2] (l0..l3); N16 = N rounded up to 16, KQp = K / 4 rounded up to a
    multiple of kq_mult, zero padded (padding channels / quads contribute exact zeros)."""
    n16 = (N + 15) // 16 * 16
    kqp = -(-(K // 4) // kq_mult) * kq_mult
    w = torch.zeros(n16, kqp * 4, dtype=torch.float32, device=wt.device)
    n = min(wt.shape[0], N)
    w[:n, :K] = wt.reshape(wt.shape[0], -1)[:n, :K].float()
    h, m, l = (t.reshape(n16, kqp, 4) for t in split_bf16x3(w))
    mh = torch.cat([m, h], dim=-1).contiguous().view(torch.int32).reshape(-1)
    lp = l.contiguous().view(torch.int32).reshape(-1)
    return torch.cat([mh, lp]).contiguous()


def gemm_weights_panel(wt: torch.Tensor) -> torch.Tensor:
    """GEMM weights [N][K] f32 (scale folded) -> the layout krrn_gemm_panel_x3_f32 reads: int32
    [N/32][K/8][384]; per (column tile nb, 8-k group g) 64 lanes x [m0..m3
    h0..h3] (256 words) then 64 lanes x [l0..l3] (128 words), lane fh*32 + nl = column 32 nb + nl,
    k = 8 g + 4 fh .. + 3. N % 32 == 0, K % 8 == 0."""
    N, K = wt.shape
    h, m, l = (t.reshape(N, K // 4, 4) for t in split_bf16x3(wt))
    mh = torch.cat([m, h], dim=-1).contiguous().view(torch.int32)             # [N][K/4][4]
    mh = mh.reshape(N // 32, 32, K // 8, 2, 4).permute(0, 2, 3, 1, 4)        # nb g fh nl 4
    lp = l.contiguous().view(torch.int32).reshape(N // 32, 32, K // 8, 2, 2).permute(0, 2, 3, 1, 4)
    return torch.cat([mh.reshape(N // 32, K // 8, 256), lp.reshape(N // 32, K // 8, 128)], dim=-1).contiguous()


def wino_eligible(spec: ConvSpec, M: int) -> bool:
    """Fused Winograd for the wide stride-1 3x3 convs (>= 32 channels in and out, >= 32k output
    pixels); the narrow HRNet branches stay on the implicit GEMM (latency-bound there)."""
    if not WINO:
        return False
    return (spec.kind == "conv" and spec.ksize == 3 and spec.stride == 1 and spec.pad == 1
            and spec.cin_p >= 32 and spec.cout >= 32 and M >= 32768)


def wino4_eligible(spec: ConvSpec, x, H: int, W: int) -> bool:
    """Winograd F(4x4, 3x3) (krrn_conv3x3_wino4_x3_f32) for the heads' wide 128 -> 128 convs: a
    wino-eligible conv with >= 64 input channels (a multiple of 8), >= 64 outputs and a map of at
    least 32 x 32, whose NHWC input is 16-byte aligned. The narrower / smaller Winograd convs (layer1
    and last_layer at S/4, 64 / 272 channels at 30 x 30) keep F(2x2): measured per shape,
    DESIGN.md section 3."""
    if not WINO4:
        return False
    return (spec.cin_p % 8 == 0 and spec.cin_p >= 64 and spec.cout >= 64 and min(H, W) >= 32
            and x.cs % 4 == 0 and x.co % 4 == 0)


def small_conv_config(M: int, ntiles: int, cin_p: int):
    """(nw, ks) for krrn_conv_small_f32 from the branch-conv sweep (profiles/bench_branch_conv.py,
    W18 at B = 64): 30x30x20 (2, 1) 17.5 us, 15x15x36 (3, 2) 12.7 us, 8x8x72 (3, 4) 12.7 us, 4x4x144
    (3, 4) 14.2 us, against 18.4 / 15.5 / 17.9 / 17.3 us for the best implicit-GEMM tile / split-K.
    Large M: whole reductions per wave; small M: the reduction split over the block's waves."""
    ks = 1 if M >= 32768 else (2 if M >= 8192 else 4)
    nw = 3 if ntiles >= 3 else ntiles
    return nw, ks


def small_conv_eligible(spec: ConvSpec, x) -> bool:
    """krrn_conv_small_f32: narrow convs whose 64-pixel blocks' input rows fit the LDS (up to 256
    physical input channels): every 3x3 / stride-1 / pad-1 conv (the HRNet branches' BasicBlocks),
    and the latency-bound 3x3 / stride-2 and 1x1 convs of the fuse layers and transitions (output
    M <= 16384 pixels or <= 32 channels; the stem and layer1's wide ones stay on the implicit GEMM)."""
    if spec.kind != "conv":
        return False
    k, st, pad = spec.ksize, spec.stride, spec.pad
    if not ((k == 3 and pad == 1 and st in (1, 2)) or (k == 1 and pad == 0 and st == 1)):
        return False
    if spec.cin_p > 256 or x.co % 4 or x.cs % 4:
        return False
    Ho, Wo = conv_out_hw(spec, x.H, x.W)
    HWo = Ho * Wo
    M = x.B * HWo
    if not (k == 3 and st == 1) and not (M <= 16384 or spec.cout <= 32):
        return False
    pitch = (spec.cin_p // 4) | 1
    rows = 0
    for p0 in range(0, min(M, 64 * HWo), 16):  # block starts repeat modulo lcm(pixb, HWo)
        p1 = min(p0 + 64, M) - 1
        bA, bB = p0 // HWo, p1 // HWo
        yA, yB = (p0 - bA * HWo) // Wo, (p1 - bB * HWo) // Wo
        r = sum(((st * yB) if b == bB else st * (Ho - 1)) + k - 1 - ((st * yA) if b == bA else 0) + 1
                for b in range(bA, bB + 1))
        rows = max(rows, r)
    return rows * (x.W + 2 * pad) * pitch * 16 <= 96 * 1024


def make_convT(convT: torch.nn.ConvTranspose2d, bn: Optional[torch.nn.Module], device,
               cin_map: Optional[List[int]] = None, cin_p: Optional[int] = None) -> ConvSpec:
    """Stride-2 ConvTranspose2d as four parity-class convolutions.

    Output row oy = 2*iy - pad + ky (+ output_padding rows at the end). For parity
    py = oy % 2, oy = 2a + py, the contributing taps satisfy ky = 2(a - iy) + py + pad,
    i.e. iy = a + (py + pad - ky) / 2 for every ky with (py + pad - ky) even.
    """
    w = convT.weight.detach().cpu()  # [cin, cout, kh, kw]
    cin, cout, kh, kw = w.shape
    assert convT.stride[0] == 2 and convT.stride[1] == 2 and kh == kw
    pad = convT.padding[0]
    if cin_map is None:
        cin_map = list(range(cin))
    cin_p = pad4(max(cin_map) + 1) if cin_p is None else cin_p
    wc = w.permute(1, 0, 2, 3)  # [cout, cin, kh, kw]
    wts, taps_all, offs = [], [], []
    for py in range(2):
        for px in range(2):
            taps_k, taps = [], []
            for ky in range(kh):
                if (py + pad - ky) % 2:
                    continue
                for kx in range(kw):
                    if (px + pad - kx) % 2:
                        continue
                    taps_k.append((ky, kx))
                    taps.append(((py + pad - ky) // 2, (px + pad - kx) // 2))
            wts.append(_pack_taps(wc, taps_k, cin_map, cin_p, cout).to(device))
            taps_all.append(taps)
            offs.append((py, px))
    scale, bias = fold_bn(cout, convT.bias, bn, device)
    return ConvSpec(wts, taps_all, offs, scale, bias, cin_p, cout, 1, "convT", kh, pad, len(cin_map))


def make_linear(weight: torch.Tensor, bias: Optional[torch.Tensor], bn: Optional[torch.nn.Module], device,
                cin_map: Optional[List[int]] = None, cin_p: Optional[int] = None) -> ConvSpec:
    """A [cout, cin] matrix (Conv1d k=1 or GCN weights^T) as a 1-tap conv spec."""
    w = weight.detach().cpu().float()
    if w.dim() == 3:
        w = w[:, :, 0]
    cout, cin = w.shape
    if cin_map is None:
        cin_map = list(range(cin))
    cin_p = pad4(max(cin_map) + 1) if cin_p is None else cin_p
    wt = _pack_taps(w[:, :, None, None], [(0, 0)], cin_map, cin_p, cout).to(device)
    scale, bias_f = fold_bn(cout, bias, bn, device)
    return ConvSpec([wt], [[(0, 0)]], [(0, 0)], scale, bias_f, cin_p, cout, 1, "conv", 1, 0, len(cin_map))
