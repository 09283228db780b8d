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
from contextlib import contextmanager
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib, knobs, ops

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
D = ctypes.c_double
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
_lib.register("krrn_gather2_add_f32", [P, P, L, I, P, P, L, I, I, I, P, P, P, I, P, L, I, I, P])
_lib.register("krrn_pnp_ransac_f32", [P, I, P, I, P, I, P, P, P, P, P, P, I, F, D, P, P, P, P, P, I, P])
_lib.register("krrn_randperm_i32", [P, U, I, I, I, P, P])
_lib.register("krrn_ransac_subsets", [P, U, I, I, I, P, P])
_lib.register("krrn_randperm_multi_i32", [P, I, P, P, P, P, P])
_lib.register("krrn_rng_advance", [P, P])
_lib.register("krrn_conv2d_group_f32", [P, I, I, P])
_lib.register("krrn_conv2d_group_x3_f32", [P, I, I, P])
_lib.register("krrn_conv2d_x3_f32", [P, I, I, I, I, I, I, I, I, I, I, P, P, P, I, I, P, P, P, I, P, I, I, P, I, I, I, I,
                                     I, I, I, I, I, I, I, P, P])
_lib.register("krrn_conv3x3_wino_f32", [P, I, I, I, I, I, I, P, I, I, P, P, P, I, I, P, I, I, I, P])
_lib.register("krrn_conv3x3_wino_x3_f32", [P, I, I, I, I, I, I, P, I, I, P, P, P, I, I, P, I, I, I, P])
_lib.register("krrn_conv3x3_wino4_x3_f32", [P, I, I, I, I, I, I, P, I, I, P, P, P, I, I, P, I, I, I, P])
_lib.register("krrn_convT_s2_x3_f32", [P, I, I, I, I, I, I, P, P, I, P, P, I, P, I, I, I, I, P])
_lib.register("krrn_conv3x3_wino_x3_head_f32", [P, I, I, I, I, I, I, P, I, P, P, P, I, I, I, P, P, I, P, P, I, P])
_lib.register("krrn_conv3x3_wino4_x3_head_f32", [P, I, I, I, I, I, I, P, I, P, P, P, I, I, I, P, P, I, P, P, I, P])
_lib.register("krrn_conv1x1_nchw_f32", [P, I, I, I, I, I, P, I, I, P, P, P, I, I, P])
_lib.register("krrn_conv1x1_nchw_x3_f32", [P, I, I, I, I, I, P, I, I, P, P, P, I, I, P])
_lib.register("krrn_conv_small_f32", [P, I, I, I, I, I, I, P, I, I, P, P, P, I, I, P, I, I, I, I, I, I, I, P])
_lib.register("krrn_blas_gemm_create", [I, I, I, I, I, I, L, L, I, I, I, I, L, L, P, P])
_lib.register("krrn_blas_gemm_run", [P, P, P, P, P, P, P, L, P])
_lib.register("krrn_blas_gemm_destroy", [P])
_lib.register("krrn_gemm_x3_f32", [P, I, I, I, I, P, P, P, I, P, I, I, I, L, L, L, P])
_lib.register("krrn_gemm_x3_gather_f32", [P, P, L, I, P, P, L, I, I, I, I, I, P, P, P, I, I, P])
_lib.register("krrn_gemm_panel_x3_f32", [P, I, I, I, I, P, P, P, I, P, I, I, I, P])


class ConvDesc(ctypes.Structure):
    """krrn_conv_desc (include/krrn_hip.h)."""
    _fields_ = [("in_", P), ("in_cs", I), ("in_co", I), ("B", I), ("Hi", I), ("Wi", I), ("cin", I), ("Hg", I),
                ("Wg", I), ("in_s", I), ("ntaps", I), ("tap_dy", I * 9), ("tap_dx", I * 9), ("wt", P), ("N", I),
                ("n_store", I), ("scale", P), ("bias", P), ("bias2", P), ("b2_div", I), ("res", P), ("res_cs", I),
                ("res_co", I), ("out", P), ("out_cs", I), ("out_co", I), ("Ho", I), ("Wo", I), ("osy", I),
                ("osx", I), ("ooy", I), ("oox", I), ("relu", I), ("out_nchw", I), ("splits", I), ("workspace", P),
                ("k_chunk", I)]

STREAM = "__stream__"


def _skey(sid: int) -> str:
    return STREAM if sid == 0 else f"__stream{sid}__"


def ptr(t: Optional[torch.Tensor]) -> P:
    return P(t.data_ptr()) if t is not None else P(0)


def h2d(t: torch.Tensor, device, dtype=None) -> torch.Tensor:
    """`t` on `device` (as `dtype`), contiguous. A host tensor bound for the GPU goes through pinned
    memory with a non-blocking copy: a copy from pageable memory is synchronous on this runtime, so it
    would stall the host until the stream drained and serialise the next batch's host-side preparation
    behind the GPU work already queued (the eval epoch's per-batch inputs, perms and metric operands).
    torch's pinned allocator keeps the staging block alive until the copy has run."""
    device = torch.device(device)
    if dtype is not None and t.dtype != dtype and t.device.type == "cpu":
        t = t.to(dtype)
    if t.device.type == "cpu" and device.type == "cuda":
        t = t.contiguous().pin_memory()
    return t.to(device=device, dtype=dtype if dtype is not None else t.dtype, non_blocking=True).contiguous()


class Late:
    """A late-bound argument: the pointer of env[key] (or env[key] itself if not a tensor)."""
    __slots__ = ("key",)

    def __init__(self, key: str):
        self.key = key


class Op:
    """One C-ABI call. `meta` carries accounting for the bench: the device kernel it launches
    ('kernel'), algorithmic FLOPs ('flops') and compulsory HBM bytes ('bytes')."""
    __slots__ = ("name", "fn", "args", "patches", "meta", "sid")

    def __init__(self, name: str, args: Sequence[Any], meta: Optional[dict] = None, sid: int = 0):
        self.name = name
        self.fn = getattr(_lib.lib(), name)
        self.args = list(args)
        self.patches: List[Tuple[int, str]] = [(i, a.key) for i, a in enumerate(self.args) if isinstance(a, Late)]
        self.meta = meta or {}
        self.sid = sid

    def __call__(self, env: Dict[str, Any]):
        args = self.args
        for i, key in self.patches:
            v = env[key]
            args[i] = P(v.data_ptr()) if isinstance(v, torch.Tensor) else v
        st = self.fn(*args)
        if st != 0:
            _lib.check(st, self.name)


class Sync:
    """Stream dependency: `dst` waits for everything enqueued on `src` so far (an event record +
    stream wait; under hipGraph capture this becomes a graph edge)."""
    __slots__ = ("src", "dst", "event", "name", "meta", "sid")

    def __init__(self, src: int, dst: int):
        self.src, self.dst = src, dst
        self.event = torch.cuda.Event() if torch.cuda.is_available() else None
        self.name, self.meta, self.sid = "sync", {}, dst

    def __call__(self, env: Dict[str, Any]):
        streams = env["__streams__"]
        if streams is None:  # serial run
            return
        self.event.record(streams[self.src])
        streams[self.dst].wait_event(self.event)


class _CaptureDeps:
    """hipStreamGetCaptureInfo_v2 + hipStreamUpdateCaptureDependencies (the HIP runtime torch uses):
    make a capturing stream depend on another capturing stream's current leaf nodes without an
    event. Side-stream-to-side-stream event waits made hipGraph capture segfault at capture end on
    this image whenever several of them crossed (profiles/hip_capture_crosswait.py, rc 139 with the
    events kept alive or not); the same dependencies as capture edges replay correctly
    (profiles/hip_capture_deps.py, round 6)."""
    _hip = None

    @classmethod
    def hip(cls):
        if cls._hip is None:
            h = ctypes.CDLL("libamdhip64.so")
            h.hipStreamGetCaptureInfo_v2.argtypes = [P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulonglong),
                                                     ctypes.POINTER(P), ctypes.POINTER(ctypes.POINTER(P)),
                                                     ctypes.POINTER(ctypes.c_size_t)]
            h.hipStreamUpdateCaptureDependencies.argtypes = [P, ctypes.POINTER(P), ctypes.c_size_t, ctypes.c_uint]
            cls._hip = h
        return cls._hip

    @classmethod
    def add(cls, src: "torch.cuda.Stream", dst: "torch.cuda.Stream") -> bool:
        """dst's next captured work depends on everything captured on src so far; False (nothing
        done) when src is not capturing."""
        h = cls.hip()
        st, cid, graph = ctypes.c_int(), ctypes.c_ulonglong(), P()
        deps, n = ctypes.POINTER(P)(), ctypes.c_size_t()
        e = h.hipStreamGetCaptureInfo_v2(P(src.cuda_stream), ctypes.byref(st), ctypes.byref(cid), ctypes.byref(graph),
                                         ctypes.byref(deps), ctypes.byref(n))
        if e != 0 or st.value != 1:  # hipStreamCaptureStatusActive
            return False
        nodes = (P * max(1, n.value))(*[deps[k] for k in range(n.value)])
        e = h.hipStreamUpdateCaptureDependencies(P(dst.cuda_stream), nodes, n.value, 0)  # hipStreamAddCaptureDependencies
        if e != 0:
            raise RuntimeError(f"hipStreamUpdateCaptureDependencies failed ({e})")
        return True


class Edge(Sync):
    """Sync between two side streams: a capture edge (_CaptureDeps) under hipGraph capture, an
    event record / wait otherwise."""
    __slots__ = ()

    def __call__(self, env: Dict[str, Any]):
        streams = env["__streams__"]
        if streams is None:  # serial run
            return
        if not _CaptureDeps.add(streams[self.src], streams[self.dst]):
            Sync.__call__(self, env)


# KRRN_DIAG_DROP=name[,name...]: leave every launch of those C-ABI entry points out of new plans.
# A what-if timing diagnostic (profiles/whatif.sh: how much the step shrinks if a kernel family
# were free); the outputs are meaningless with it set, and nothing in the package sets it.
_DIAG_DROP = frozenset(filter(None, knobs.text("KRRN_DIAG_DROP").split(",")))
# KRRN_PLAN_STREAMS=1 (default): a plan captured into a hipGraph keeps its side streams (graph
# branches); 0 = captured serially. KRRN_STREAMS=1 (default): the two-slot pipeline's stages and
# concurrent micro-batches replay side by side on two streams; 0 = one after the other. Rounds 3-4
# kept it off while two graphs side by side gave a different level-0 surface-conv output; the cause
# was a packed-FP32 VALU result going wrong beside the split-bf16 Winograd, and the library is now
# built without packed-FP32 ops
PLAN_STREAMS = knobs.flag("KRRN_PLAN_STREAMS")
STREAMS = knobs.flag("KRRN_STREAMS")


class Plan:
    """An ordered launch list plus the workspaces it owns.

    Ops are tagged with a stream id (`on_stream`); id 0 is the caller's current stream and ids
    1.. are plan-owned side streams, ordered by explicit `fork` / `join` points. Independent
    HRNet branches and head towers use this to run concurrently (one small conv cannot fill 256
    CUs; four of them side by side fill more).

    `run()` is serial by default (everything on the caller's stream); the side streams are used
    only with `run(serial=False)` under hipGraph capture, where every fork / join becomes a graph
    edge (KRRN_PLAN_STREAMS=0 makes captured plans serial too). The mismatches that led to this
    (round 2: eager plans on ~7 streams; round 3: two graphs side by side) were a packed-FP32 VALU
    result going wrong while the split-bf16 Winograd ran on the same CU, not a missing dependency
    (serial write audit clean, the kernel's inputs, LDS and arguments identical); the
    library is built without packed-FP32 ops since round 4."""

    def __init__(self, device: torch.device):
        self.device = device
        self.ops: List[Any] = []
        self.buffers: List[torch.Tensor] = []  # keep-alive
        self.cur = 0
        self.nstreams = 1
        self._side: List[torch.cuda.Stream] = []
        self._scratch: Dict[Tuple[int, int], torch.Tensor] = {}
        self._packed: Dict[tuple, torch.Tensor] = {}  # packed GEMM weights, shared by repeated GEMMs

    def buf(self, shape, dtype=torch.float32, zero: bool = True) -> torch.Tensor:
        t = (torch.zeros if zero else torch.empty)(tuple(shape), dtype=dtype, device=self.device)
        self.buffers.append(t)
        return t

    def scratch(self, nfloats: int, slot: int = 0) -> torch.Tensor:
        """A workspace for the current stream (ops on one stream run in order, so they can share
        it; a larger request allocates a larger one, earlier ops keep theirs). `slot` separates
        the problems of one grouped launch, which run concurrently."""
        key = (self.cur, slot)
        ws = self._scratch.get(key)
        if ws is None or ws.numel() < nfloats:
            ws = self.buf((max(nfloats, 1 << 20),), zero=False)
            self._scratch[key] = ws
        return ws

    def add(self, name: str, *args, meta: Optional[dict] = None):
        if _DIAG_DROP and name in _DIAG_DROP:
            return  # what-if timing diagnostic only (results are wrong): see _DIAG_DROP
        self.ops.append(Op(name, list(args) + [Late(_skey(self.cur))], meta, self.cur))

    @contextmanager
    def on_stream(self, sid: int):
        prev, self.cur = self.cur, sid
        self.nstreams = max(self.nstreams, sid + 1)
        try:
            yield
        finally:
            self.cur = prev

    def fork(self, sids: Sequence[int]):
        """Side streams `sids` wait for all work so far on stream 0."""
        for s in sids:
            if s != 0:
                self.ops.append(Sync(0, s))

    def join(self, sids: Sequence[int]):
        """Stream 0 waits for all work so far on side streams `sids`."""
        for s in sids:
            if s != 0:
                self.ops.append(Sync(s, 0))

    def sync(self, src: int, dst: int):
        """Stream `dst` waits for all work so far on stream `src`."""
        if src != dst:
            self.nstreams = max(self.nstreams, src + 1, dst + 1)
            self.ops.append(Sync(src, dst))

    def edge(self, src: int, dst: int):
        """Stream `dst` waits for all work so far on stream `src`, as a capture edge (Edge): for
        dependencies between two side streams."""
        if src != dst:
            self.nstreams = max(self.nstreams, src + 1, dst + 1)
            self.ops.append(Edge(src, dst))

    def side_streams(self) -> List[torch.cuda.Stream]:
        while len(self._side) < self.nstreams - 1:
            self._side.append(torch.cuda.Stream(self.device))
        return self._side

    def _streams(self, env: Dict[str, Any], serial: bool):
        main = torch.cuda.current_stream(self.device)
        self.side_streams()
        streams = [main] + self._side
        for sid in range(self.nstreams):
            env[_skey(sid)] = P((main if serial else streams[sid]).cuda_stream)
        env["__streams__"] = None if serial else streams
        return main

    def run(self, env: Dict[str, Any], serial: bool = True):
        serial = serial or not PLAN_STREAMS
        self._streams(env, serial)
        for op in self.ops:
            op(env)

    def __len__(self):
        return len(self.ops)

    def kernels(self) -> List[Op]:
        return [op for op in self.ops if isinstance(op, Op)]

    def run_timed(self, env: Dict[str, Any]) -> List[Tuple[Op, float]]:
        """Run once serially with a HIP event pair around every launch (on the launch stream);
        returns (op, device ms) per kernel launch. Diagnostic only: the host-side recording
        makes this slower than a plain/graph run."""
        stream = self._streams(env, serial=True)
        kops = self.kernels()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(kops) + 1)]
        evs[0].record(stream)
        for i, op in enumerate(kops):
            op(env)
            evs[i + 1].record(stream)
        stream.synchronize()
        return [(op, evs[i].elapsed_time(evs[i + 1])) for i, op in enumerate(kops)]


def conv_tile(M: int, N: int, K: int = 1024, nchw: bool = False) -> int:
    """Tile choice for krrn_conv2d_f32 from the measured menu (scratch/convbench.py on MI355X,
    graph-replayed, buffer-load staging): 64x64x32 (4-5 waves/SIMD) is best or within 3% on
    every wide layer (S=120 head conv 119 TF vs 121 for hipBLASLt's f32 GEMM of the same
    shape; TBase conv1 118 TF); 128x32x32 with 4 waves along M for N <= 32 (HRNet branch 0 and
    its transitions: 51 vs 33 TF). NCHW-output heads use 128x32x32 up to N = 96 (the head
    logits: N = 72 pads to 3 x 32 instead of 2 x 64), 64x64x16 above."""
    if nchw:
        return 6 if N <= 96 else 3
    if N <= 32:
        return 6
    return 8


TILE_SHAPES = {1: (128, 128, 16), 2: (128, 64, 16), 3: (64, 64, 16), 4: (128, 128, 32), 5: (256, 32, 16),
               6: (128, 32, 32), 7: (128, 64, 32), 8: (64, 64, 32)}


SPLITK = knobs.flag("KRRN_SPLITK")
SPLITK_TILES = 256  # split only launches with fewer tiles
SPLITK_NKT = 8      # ... and at least this many k-tiles
SPLITK_PER = 4      # k-tiles per split at least


def conv_splits(M: int, N: int, K: int, tile: int) -> int:
    """Split-K factor: layers with fewer than 256 output tiles (the 8x8 / 4x4 HRNet branches, M =
    B*64 / B*16) and a deep K get their k-tiles split across blockIdx.y until ~512 workgroups
    exist, keeping >= 4 k-tiles per split."""
    BM, BN, BK = TILE_SHAPES[tile]
    cd = lambda a, b: (a + b - 1) // b  # noqa: E731
    tiles = cd(M, BM) * cd(N, BN)
    nkt = cd(K, BK)
    if tiles >= SPLITK_TILES or nkt < SPLITK_NKT or N % 4 or not SPLITK:
        return 1
    return max(1, min(cd(512, tiles), nkt // SPLITK_PER, 16))


CONV_KERNELS = {1: "conv_gemm_f32<128,128,16>", 2: "conv_gemm_f32<128,64,16>", 3: "conv_gemm_f32<64,64,16>",
                4: "conv_gemm_f32<128,128,32>", 5: "conv_gemm_f32<256,32,16>", 6: "conv_gemm_f32<128,32,32>",
                7: "conv_gemm_f32<128,64,32>", 8: "conv_gemm_f32<64,64,32>"}


def _iarr(vals):
    arr = (ctypes.c_int * 9)()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr


# split-bf16 implicit GEMM (krrn_conv2d_x3_f32): 128x64x16 tiles for N > 32, no split-K
# (profiles/bench_conv_x3.py, B = 64: 3x3 / s2 64 -> 64 at 120 px 185 us against the f32 kernel's
# best 206; the 64x64x32 tile is slower in x3: 245 us, its 32x32 wave tiles LDS-bound)
X3_TILE = 2


def add_conv(plan: Plan, *, x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s, taps, wt, N, n_store, scale, bias,
             bias2=None, b2_div=1, res=None, res_cs=0, res_co=0, out, out_cs, out_co, Ho, Wo, osy=1, osx=1, ooy=0,
             oox=0, relu=False, nchw=False, cin=None, cout=None, tag="", tile=None, splits=None, wt3=None):
    """Append one krrn_conv2d_f32 launch, or krrn_conv2d_x3_f32 (split-bf16 operands, f32 accuracy)
    when `wt3` (ops.conv_weights_x3 of the weights) is given and the tile allows. Pointers are
    ctypes values (see `ptr`). cin/cout are the logical channel counts used for the algorithmic
    FLOP count 2*cin*cout*ntaps*M."""
    M = B * Hg * Wg
    K = cin_p * len(taps)
    tile_req = tile
    tile = conv_tile(M, N, K, nchw) if tile is None else tile
    if splits is None:
        splits = 1 if nchw else conv_splits(M, N, K, tile)
    ws = plan.scratch(splits * M * N) if splits > 1 else None
    cin = cin_p if cin is None else cin
    cout = n_store if cout is None else cout
    flops = 2.0 * cin * cout * len(taps) * M
    kname = CONV_KERNELS[tile] + (",nchw" if nchw else "") + (",splitk" if splits > 1 else "")
    if wt3 is not None and not nchw and N > 32 and splits == 1:
        tile = X3_TILE if tile_req is None else tile_req
        # matrix pipe: 6 bf16 term products per f32 product at 16x the f32 rate (f32-MFMA time)
        kname = CONV_KERNELS[tile]
        plan.add("krrn_conv2d_x3_f32", x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s, len(taps),
                 _iarr([t[0] for t in taps]), _iarr([t[1] for t in taps]), wt3, N, n_store, scale, bias,
                 bias2 if bias2 is not None else P(0), b2_div, res if res is not None else P(0), res_cs, res_co, out,
                 out_cs, out_co, Ho, Wo, osy, osx, ooy, oox, int(relu), tile, splits, ptr(ws),
                 meta=dict(kernel=kname.replace("conv_gemm_f32", "conv_gemm_x3"), flops=flops, tag=tag, M=M, N=N,
                           K=K, splits=splits, mfma_flops=2.0 * M * N * K * 6 / 16,
                           mfma_bf16_flops=2.0 * M * N * K * 6))
        return
    plan.add("krrn_conv2d_f32", x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s, len(taps), _iarr([t[0] for t in taps]),
             _iarr([t[1] for t in taps]), wt, N, n_store, scale, bias, bias2 if bias2 is not None else P(0), b2_div,
             res if res is not None else P(0), res_cs, res_co, out, out_cs, out_co, Ho, Wo, osy, osx, ooy, oox,
             int(relu), int(nchw), tile, splits, ptr(ws),
             meta=dict(kernel=kname, flops=flops, tag=tag, M=M, N=N, K=K, splits=splits))


GROUP_TILE = 6


def conv_desc(*, x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s, taps, wt, N, n_store, scale, bias, res=None,
              res_cs=0, res_co=0, out, out_cs, out_co, Ho, Wo, osy=1, osx=1, ooy=0, oox=0, relu=False,
              splits=1, ws=None, k_chunk=0) -> ConvDesc:
    d = ConvDesc()
    d.in_, d.in_cs, d.in_co, d.B, d.Hi, d.Wi, d.cin, d.Hg, d.Wg, d.in_s = x, x_cs, x_co, B, Hi, Wi, cin_p, Hg, Wg, in_s
    d.ntaps = len(taps)
    for i, (dy, dx) in enumerate(taps):
        d.tap_dy[i], d.tap_dx[i] = dy, dx
    d.wt, d.N, d.n_store, d.scale, d.bias, d.bias2, d.b2_div = wt, N, n_store, scale, bias, P(0), 1
    d.res = res if res is not None else P(0)
    d.res_cs, d.res_co = res_cs, res_co
    d.out, d.out_cs, d.out_co, d.Ho, d.Wo = out, out_cs, out_co, Ho, Wo
    d.osy, d.osx, d.ooy, d.oox, d.relu, d.out_nchw = osy, osx, ooy, oox, int(relu), 0
    d.splits, d.workspace = splits, (ws if ws is not None else P(0))
    d.k_chunk = k_chunk
    return d


def add_conv_group(plan: Plan, problems: List[dict], tile: int = None, tag: str = "group", x3: bool = False):
    """One krrn_conv2d_group_f32 launch over up to 4 independent convs (dicts of conv_desc
    keyword arguments plus 'cin' / 'cout' logical channels for the FLOP count), or
    krrn_conv2d_group_x3_f32 (x3: every problem's `wt` is ops.conv_weights_x3 chains)."""
    tile = GROUP_TILE if tile is None else tile
    n = len(problems)
    arr = (ConvDesc * n)()
    flops = 0.0
    nsplit = 1
    shapes = []
    for q, pr in enumerate(problems):
        pr = dict(pr)
        cin, cout = pr.pop("cin"), pr.pop("cout")
        M = pr["B"] * pr["Hg"] * pr["Wg"]
        K = pr["cin_p"] * len(pr["taps"])
        sp = conv_splits(M, pr["N"], K, tile)
        ws = ptr(plan.scratch(sp * M * pr["N"], slot=q)) if sp > 1 else None
        arr[q] = conv_desc(**pr, splits=sp, ws=ws)
        flops += 2.0 * cin * cout * len(pr["taps"]) * M
        nsplit = max(nsplit, sp)
        shapes.append((M, pr["N"], K, sp))
    plan.buffers.append(arr)
    meta = dict(kernel=f"conv_group{'_x3' if x3 else ''}<{','.join(map(str, TILE_SHAPES[tile]))}>", flops=flops,
                tag=tag, M=shapes[0][0], N=shapes[0][1], K=shapes[0][2], splits=nsplit, shapes=shapes)
    if x3:
        pipe = sum(2.0 * M * N * K for M, N, K, _ in shapes)
        meta.update(mfma_flops=pipe * 6 / 16, mfma_bf16_flops=pipe * 6)
    plan.add("krrn_conv2d_group_x3_f32" if x3 else "krrn_conv2d_group_f32", ctypes.cast(arr, P), n, tile, meta=meta)


BLAS = knobs.flag("KRRN_BLAS")
BLAS_MAX_WS = 64 << 20
# plain GEMMs with K >= GEMM_X3_MINK on gemm_x3.hip (split-bf16), the rest on hipBLASLt: measured
# (profiles/bench_gemm.py, MI355X) 10-18 % faster at K = 256..1024, 10 % slower at K = 128 (the
# level-0 GCN GEMMs: 198 vs 180 us, output-write-bound) and slower at layer1's K = 64 (all
# eligible GEMMs on gemm_x3: 1.98 vs 1.77 ms of GEMMs per step)
GEMM_X3 = knobs.flag("KRRN_GEMM_X3")
# short-K GEMMs (K = 64 / 128, N % 32 == 0, one row group) on the A-stationary split-bf16 kernel
# (gemm_panel.hip): the level-0 / level-1 GCN GEMMs, whose 262 MB output makes them write streams
GEMM_PANEL = knobs.flag("KRRN_GEMM_PANEL")
GEMM_X3_MINK = 256


class _BlasPlan:
    """Owns one krrn_blas_gemm plan (destroyed with the launch plan that keeps it)."""

    def __init__(self, handle):
        self.handle = handle

    def __del__(self):
        try:
            if self.handle:
                _lib.lib().krrn_blas_gemm_destroy(self.handle)
        except Exception:  # interpreter shutdown
            pass


def add_gemm(plan: Plan, *, a: torch.Tensor, a_off: int, lda: int, M: int, wt: torch.Tensor, K: int, N: int,
             scale: Optional[torch.Tensor], bias: Optional[torch.Tensor], out: torch.Tensor, ldo: int, relu: bool,
             res: Optional[torch.Tensor] = None, ldr: int = 0, batch: int = 1, a_grp: int = 0, o_grp: int = 0,
             r_grp: int = 0, cin: Optional[int] = None, cout: Optional[int] = None, tag: str = "gemm",
             require_x3: bool = False, blas_ok: bool = True) -> bool:
    """Append a plain GEMM out[m, n] = act(scale[n] * (A[m] . wt[n]) + bias[n] (+ res[m, n])) on hipBLASLt
    (krrn_blas_gemm_*; scale folded into the weights). Returns False when hipBLASLt is disabled
    (KRRN_BLAS=0) or rejects the problem: the caller then emits its own kernel. Short-K GEMMs go to
    the A-stationary split-bf16 kernel and K >= 256 ones to gemm_x3 first (own kernels).
    require_x3: only gemm_x3 will do (its ldr = 0 per-group row broadcast); False if ineligible.
    blas_ok=False: own kernels only (False instead of a hipBLASLt plan).
    A K = 128 GEMM with a residual is not taken by the panel kernel (its 128-VGPR activation chain
    leaves no room for the residual tile; krrn_gemm_panel_x3_f32 returns KRRN_EUNSUPPORTED), nor is
    one wider than the kernel's 2048-column bias stage (KRRN_ESHAPE)."""
    dev = plan.device
    w = wt.reshape(N, -1)[:, :K].float()
    if scale is not None:
        w = w * scale.reshape(N, 1).to(w.device)
    w = w.contiguous()
    wkey = (wt.data_ptr(), scale.data_ptr() if scale is not None else 0, K, N)

    def packed(kind: str, fn):
        """The kernel's packed weights, built once per (weights, scale, kind) in a plan: a GEMM
        repeated over row chunks (the fusion's level-0 crop chunks) shares one copy."""
        key = wkey + (kind,)
        if key not in plan._packed:
            plan._packed[key] = fn(w)
            plan.buffers.append([plan._packed[key], bias])
        return plan._packed[key]
    flops = 2.0 * (cin or K) * (cout or N) * M * batch
    if GEMM_PANEL and not require_x3 and K in (64, 128) and N % 32 == 0 and N <= 2048 and batch == 1 \
            and lda % 4 == 0 and a_off % 4 == 0 and not (K == 128 and res is not None):
        wp = packed("panel", ops.gemm_weights_panel)
        csplit = 1
        tiles = N // 32
        if K == 128:
            # the level-0 / level-1 GCN GEMMs (128-row blocks, two per CU): about 16 column tiles per
            # block and at least 512 blocks; measured (profiles/bench_fusion_kernels.py, round 4) level 0
            # (M = 64000) 124 us at csplit 2 against 132 at 1, level 1 (M = 16000) 35 us at 4 against 42 at 8
            blocks = (M + 127) // 128
            while tiles % (2 * csplit) == 0 and (tiles // csplit > 16 or
                                                 (blocks * csplit < 512 and tiles // csplit >= 16)):
                csplit *= 2
        else:
            rows = (M + 255) // 256
            while rows * csplit < 256 and tiles % (2 * csplit) == 0:  # fill the chip: >= 256 blocks
                csplit *= 2
        plan.add("krrn_gemm_panel_x3_f32", P(a.data_ptr() + 4 * a_off), lda, M, K, N, ptr(wp), ptr(bias), ptr(res),
                 ldr, ptr(out), ldo, int(relu), csplit,
                 meta=dict(kernel="gemm_panel_x3", flops=flops, tag=tag, M=M, N=N, K=K, splits=csplit,
                           mfma_flops=2.0 * M * N * K * 6 / 16, mfma_bf16_flops=2.0 * M * N * K * 6,
                           bytes=4.0 * (M * K + M * N)))
        return True
    if GEMM_X3 and K >= GEMM_X3_MINK and K % 32 == 0 and N % 128 == 0 and lda % 4 == 0 and ldo % 4 == 0 and a_off % 4 == 0 \
            and (res is None or ldr % 4 == 0):
        # own split-bf16 GEMM (gemm_x3.hip): 6 bf16 term products per f32 product
        w3 = packed("x3", ops.gemm_weights_x3)
        plan.add("krrn_gemm_x3_f32", P(a.data_ptr() + 4 * a_off), lda, M, K, N, ptr(w3), ptr(bias), ptr(res), ldr,
                 ptr(out), ldo, int(relu), batch, a_grp, o_grp, r_grp,
                 meta=dict(kernel="gemm_x3", flops=flops, tag=tag, M=M * batch, N=N, K=K, splits=1,
                           mfma_flops=2.0 * M * batch * N * K * 6 / 16, mfma_bf16_flops=2.0 * M * batch * N * K * 6))
        return True
    if not BLAS or require_x3 or not blas_ok:
        return False
    h = ctypes.c_void_p()
    wsb = ctypes.c_longlong()
    st = _lib.lib().krrn_blas_gemm_create(M, N, K, lda, ldo, batch, a_grp, o_grp, int(bias is not None), int(relu),
                                          int(res is not None), ldr, r_grp, BLAS_MAX_WS, ctypes.byref(h),
                                          ctypes.byref(wsb))
    if st != 0:
        return False
    owner = _BlasPlan(h)
    ws = plan.buf((max(int(wsb.value), 16),), torch.uint8, zero=False)
    plan.buffers.append([owner, w, bias])
    a_ptr = P(a.data_ptr() + 4 * a_off)
    plan.add("krrn_blas_gemm_run", h, a_ptr, ptr(w), ptr(bias), ptr(res), ptr(out), ptr(ws), int(wsb.value),
             meta=dict(kernel="hipblaslt_gemm_f32", flops=2.0 * (cin or K) * (cout or N) * M * batch, tag=tag,
                       M=M * batch, N=N, K=K, splits=1))
    return True
