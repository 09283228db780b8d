"""A tiny launch-list runtime over libkrrn_hip.so.

A model "plan" is compiled once per input shape into a flat list of C-ABI calls whose
arguments are pre-built ctypes values (device pointers of plan-owned workspaces, sizes,
folded weights). Running the plan is one ctypes call per kernel with no per-call Python
arithmetic; the only late-bound arguments are the HIP stream and user-supplied tensors,
patched from an environment dict. Because every buffer pointer is fixed, a plan can be
captured once into a hipGraph (torch.cuda.CUDAGraph drives HIP stream capture) and
replayed for the steady-state loop.
"""
from __future__ import annotations

import ctypes
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
L = ctypes.c_longlong
U = ctypes.c_uint

# C-ABI signatures (include/krrn_hip.h); every function returns int status.
_lib.register("krrn_knn_f32", [P, L, I, I, P, P, L, I, I, I, I, I, I, I, P, P])
_lib.register("krrn_gcn_conv_f32", [P, I, I, P, L, I, I, P, I, I, P, P, P, I, P, L, I, I, P])
_lib.register("krrn_pool_max_f32", [P, I, I, P, L, I, I, P, L, I, I, P])
_lib.register("krrn_resize_bilinear_f32", [P, I, I, I, I, I, I, P, I, I, I, I, P, I, I, I, I, P])
_lib.register("krrn_add_relu_f32", [P, I, I, P, I, I, P, I, I, L, I, I, P])
_lib.register("krrn_nchw_to_nhwc_f32", [P, I, I, I, I, P, I, I, P])
_lib.register("krrn_heads_select_f32", [P, I, I, P, I, P, P, P, I, I, I, P])
_lib.register("krrn_points_gather_f32", [P, P, P, P, I, I, I, I, P, P])
_lib.register("krrn_gather_rows_f32", [P, I, L, I, P, L, I, P, L, I, I, I, P])
_lib.register("krrn_tbase_tail_f32", [P, I, I, I, P, P, P, P, P, P])
_lib.register("krrn_pnp_ransac_f32", [P, I, P, I, P, I, P, P, P, P, P, P, I, F, P, P, P, P, P, I, P])
_lib.register("krrn_randperm_i32", [P, U, I, I, I, P, P])
_lib.register("krrn_ransac_subsets", [P, U, I, I, I, P, P])
_lib.register("krrn_rng_advance", [P, P])

STREAM = "__stream__"


def ptr(t: Optional[torch.Tensor]) -> P:
    return P(t.data_ptr()) if t is not None else P(0)


class Late:
    """A late-bound argument: the pointer of env[key] (or env[key] itself if not a tensor)."""
    __slots__ = ("key",)

    def __init__(self, key: str):
        self.key = key


class Op:
    """One C-ABI call. `meta` carries accounting for the bench: the device kernel it launches
    ('kernel'), algorithmic FLOPs ('flops') and compulsory HBM bytes ('bytes')."""
    __slots__ = ("name", "fn", "args", "patches", "meta")

    def __init__(self, name: str, args: Sequence[Any], meta: Optional[dict] = None):
        self.name = name
        self.fn = getattr(_lib.lib(), name)
        self.args = list(args)
        self.patches: List[Tuple[int, str]] = [(i, a.key) for i, a in enumerate(self.args) if isinstance(a, Late)]
        self.meta = meta or {}

    def __call__(self, env: Dict[str, Any]):
        args = self.args
        for i, key in self.patches:
            v = env[key]
            args[i] = P(v.data_ptr()) if isinstance(v, torch.Tensor) else v
        st = self.fn(*args)
        if st != 0:
            _lib.check(st, self.name)


class Plan:
    """An ordered launch list plus the workspaces it owns."""

    def __init__(self, device: torch.device):
        self.device = device
        self.ops: List[Op] = []
        self.buffers: List[torch.Tensor] = []  # keep-alive

    def buf(self, shape, dtype=torch.float32, zero: bool = True) -> torch.Tensor:
        t = (torch.zeros if zero else torch.empty)(tuple(shape), dtype=dtype, device=self.device)
        self.buffers.append(t)
        return t

    def add(self, name: str, *args, meta: Optional[dict] = None):
        self.ops.append(Op(name, list(args) + [Late(STREAM)], meta))

    def run(self, env: Dict[str, Any]):
        env[STREAM] = P(torch.cuda.current_stream(self.device).cuda_stream)
        for op in self.ops:
            op(env)

    def __len__(self):
        return len(self.ops)

    def run_timed(self, env: Dict[str, Any]) -> List[float]:
        """Run once with a HIP event pair around every launch (on the launch stream);
        returns per-op device milliseconds. Diagnostic only (events serialise nothing, but the
        host-side recording makes this slower than a plain/graph run)."""
        stream = torch.cuda.current_stream(self.device)
        env[STREAM] = P(stream.cuda_stream)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(self.ops) + 1)]
        evs[0].record(stream)
        for i, op in enumerate(self.ops):
            op(env)
            evs[i + 1].record(stream)
        stream.synchronize()
        return [evs[i].elapsed_time(evs[i + 1]) for i in range(len(self.ops))]


def conv_tile(M: int, N: int, K: int = 1024, nchw: bool = False) -> int:
    """Tile choice for krrn_conv2d_f32 from the measured menu (scratch/convbench.py on MI355X,
    graph-replayed): 128x128x32 only for very large, deep GEMMs (>= 2048 tiles, K >= 512: the
    S=120 head convs 103 TF, TBase conv1 104 TF); 128x32x32 with 4 waves along M for N <= 32
    (HRNet branch 0: 22 vs 15 TF for 64x64); 64x64x32 otherwise (69 TF on layer1 3x3 vs 61)."""
    cd = lambda a, b: (a + b - 1) // b  # noqa: E731
    if nchw:
        return 1 if cd(M, 128) * cd(N, 128) >= 512 else 3
    if N <= 32:
        return 6
    if N >= 128 and K >= 512 and cd(M, 128) * cd(N, 128) >= 2048:
        return 4
    return 8


CONV_KERNELS = {1: "conv_gemm_f32<128,128,16>", 2: "conv_gemm_f32<128,64,16>", 3: "conv_gemm_f32<64,64,16>",
                4: "conv_gemm_f32<128,128,32>", 5: "conv_gemm_f32<256,32,16>", 6: "conv_gemm_f32<128,32,32>",
                7: "conv_gemm_f32<128,64,32>", 8: "conv_gemm_f32<64,64,32>"}


def _iarr(vals):
    arr = (ctypes.c_int * 9)()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


def add_conv(plan: Plan, *, x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s, taps, wt, N, n_store, scale, bias,
             bias2=None, b2_div=1, res=None, res_cs=0, res_co=0, out, out_cs, out_co, Ho, Wo, osy=1, osx=1, ooy=0,
             oox=0, relu=False, nchw=False, cin=None, cout=None, tag="", tile=None):
    """Append one krrn_conv2d_f32 launch. Pointers are ctypes values (see `ptr`). cin/cout are the
    logical channel counts used for the algorithmic FLOP count 2*cin*cout*ntaps*M."""
    M = B * Hg * Wg
    tile = conv_tile(M, N, cin_p * len(taps), nchw) if tile is None else tile
    cin = cin_p if cin is None else cin
    cout = n_store if cout is None else cout
    flops = 2.0 * cin * cout * len(taps) * M
    plan.add("krrn_conv2d_f32", x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s, len(taps), _iarr([t[0] for t in taps]),
             _iarr([t[1] for t in taps]), wt, N, n_store, scale, bias, bias2 if bias2 is not None else P(0), b2_div,
             res if res is not None else P(0), res_cs, res_co, out, out_cs, out_co, Ho, Wo, osy, osx, ooy, oox,
             int(relu), int(nchw), tile,
             meta=dict(kernel=CONV_KERNELS[tile] + (",nchw" if nchw else ""), flops=flops, tag=tag, M=M, N=N,
                       K=cin_p * len(taps)))
