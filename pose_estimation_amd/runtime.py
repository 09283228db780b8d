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
_lib.register("krrn_pnp_ransac_f32", [P, I, P, I, P, I, P, P, P, P, P, P, I, F, P, P, P, P, I, P])
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
    __slots__ = ("name", "fn", "args", "patches")

    def __init__(self, name: str, args: Sequence[Any]):
        self.name = name
        self.fn = getattr(_lib.lib(), name)
        self.args = list(args)
        self.patches: List[Tuple[int, str]] = [(i, a.key) for i, a in enumerate(self.args) if isinstance(a, Late)]

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

    def add(self, name: str, *args):
        self.ops.append(Op(name, list(args) + [Late(STREAM)]))

    def run(self, env: Dict[str, Any]):
        env[STREAM] = P(torch.cuda.current_stream(self.device).cuda_stream)
        for op in self.ops:
            op(env)

    def __len__(self):
        return len(self.ops)
