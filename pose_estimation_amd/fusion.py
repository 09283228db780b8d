"""3D-GCN RGB/point fusion of KRRN (FusionNetLite, lib/network/point/fusion.py:137-240 and
lib/network/point/gcn3d.py:15-242), MI355X execution.

Parameter containers keep the reference names (`fusion.conv_1_v.weights`, `.bias`,
`.directions`, `fusion.bn1_v.*`, `fusion.conv_4.*`, ...). `build_fusion_plan` emits:

  kNN (krrn_knn_f32, no N x N matrix)            gcn3d.get_neighbor_index / get_nearest_index
  Conv_surface            -> krrn_gcn_conv_f32 (no Y)
  Conv_layer/_fuse_layer  -> `feature_map @ weights + bias` on the f32 MFMA GEMM, then
                             krrn_gcn_conv_f32 (gather + theta + max_k + sum_s + centre,
                             + the BN1d/ReLU that FusionNetLite wraps around it)
  Pool_layer              -> kNN(k=4) only at the randperm rows + krrn_pool_max_f32 +
                             krrn_gather_rows_f32 for the sampled vertices
  final concat            -> three krrn_gather_rows_f32 launches into [B, N, 1280]

Reference quirks reproduced (SURVEY.md §7 hard part 3): each branch pool draws its own
permutation but the v-branch graph idx1 is used for the x/n branches; feat_1 (level 0, N rows)
is indexed by pool-1 nearest indices < N/4; fm_pool_1 is never needed (only its permutation
is consumed); the level-2 kNN runs on the 9-D pooled features; conv_4/conv_5 have no
activation.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import knobs, ops
from .runtime import Late, Plan, add_conv, add_gemm, ptr


class Conv_surface(nn.Module):  # noqa: N801 (reference class name, gcn3d.py:72)
    def __init__(self, kernel_num, support_num):
        super().__init__()
        self.kernel_num = kernel_num
        self.support_num = support_num
        self.directions = nn.Parameter(torch.empty(3, support_num * kernel_num))
        stdv = 1.0 / math.sqrt(support_num * kernel_num)
        nn.init.uniform_(self.directions, -stdv, stdv)


class Conv_layer(nn.Module):  # noqa: N801 (gcn3d.py:115)
    dim = 3

    def __init__(self, in_channel, out_channel, support_num):
        super().__init__()
        self.in_channel, self.out_channel, self.support_num = in_channel, out_channel, support_num
        self.weights = nn.Parameter(torch.empty(in_channel, (support_num + 1) * out_channel))
        self.bias = nn.Parameter(torch.empty((support_num + 1) * out_channel))
        self.directions = nn.Parameter(torch.empty(self.dim, support_num * out_channel))
        stdv = 1.0 / math.sqrt(out_channel * (support_num + 1))
        for p in (self.weights, self.bias, self.directions):
            nn.init.uniform_(p, -stdv, stdv)


class Conv_fuse_layer(Conv_layer):  # noqa: N801 (gcn3d.py:167), 9-D directions
    dim = 9


class Pool_layer(nn.Module):  # noqa: N801 (gcn3d.py:218)
    def __init__(self, pooling_rate: int = 4, neighbor_num: int = 4):
        super().__init__()
        self.pooling_rate = pooling_rate
        self.neighbor_num = neighbor_num


class FusionNetLite(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.neighbor_num = cfg.Module.GCN3D.GCN_N_NUM
        self.support_num = cfg.Module.GCN3D.GCN_SUP_NUM
        self.num_cls = cfg.Module.NUM_CLS
        S = self.support_num
        for br in ("v", "x", "n"):
            setattr(self, f"conv_0_{br}", Conv_surface(128, S))
            setattr(self, f"conv_1_{br}", Conv_layer(128, 128, S))
            setattr(self, f"pool_1_{br}", Pool_layer(4, 4))
            setattr(self, f"conv_2_{br}", Conv_layer(128, 128, S))
            setattr(self, f"bn1_{br}", nn.BatchNorm1d(128))
            setattr(self, f"bn2_{br}", nn.BatchNorm1d(128))
        self.pool_1 = Pool_layer(4, 4)
        self.pool_2 = Pool_layer(4, 4)
        self.conv_4 = Conv_fuse_layer(384, 512, S)
        self.conv_5 = Conv_fuse_layer(512, 512, S)



FEAT_SID = 4  # plan stream of the materialised output concat (joined by the caller)
# crops per chunk of the level-0 GEMM + gather-conv (0: the whole batch in one launch each)
FUSION_CHUNK = knobs.integer("KRRN_FUSION_CHUNK")

def level_sizes(N: int, k0: int):
    N1 = int(N / 4)
    N2 = int(N1 / 4)
    k1 = min(k0, N1 // 8)
    k2 = min(k0, N2 // 8)
    return N1, N2, k1, k2


def _dn(directions: torch.Tensor, device) -> torch.Tensor:
    # F.normalize(self.directions, dim=0) (gcn3d.py:104, 145, 197), evaluated once at plan time
    return F.normalize(directions.detach().float().cpu(), dim=0).contiguous().to(device)


def _bn1d(bn: nn.BatchNorm1d, device):
    s = (bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps))
    b = bn.bias.detach().double() - bn.running_mean.detach().double() * s
    return s.float().to(device), b.float().to(device)


class _Emit:
    """The fusion's launch helpers (kNN, gather-conv, GEMM) bound to one plan and batch."""

    def __init__(self, fu: FusionNetLite, plan: Plan, B: int, keep: list):
        self.plan, self.B, self.dev, self.S, self.keep = plan, B, plan.device, fu.support_num, keep
        self._lin: dict = {}

    def knn(self, q, q_bs, q_st, nq, qidx, c, c_bs, c_st, nc, d, k, drop, mode, out):
        self.plan.add("krrn_knn_f32", q, q_bs, q_st, nq, qidx, c, c_bs, c_st, nc, d, k, drop, mode, self.B, ptr(out))

    def gcn(self, idx, n, k, v, v_bs, d, dn, C, Y, bn, relu, out, o_bs, o_st, Bc=None, v_st=9):
        self.keep.append(dn)
        s, b = (None, None) if bn is None else bn
        self.keep.extend([s, b])
        self.plan.add("krrn_gcn_conv_f32", ptr(idx), n, k, v, v_bs, v_st, d, ptr(dn), self.S, C, ptr(Y), ptr(s), ptr(b),
                      int(relu), out, o_bs, o_st, self.B if Bc is None else Bc)

    def gemm(self, a, a_cs, a_co, M, layer: "Conv_layer", out):
        # one spec per layer: a GEMM repeated over crop chunks shares its weights (and add_gemm its
        # packed copy)
        spec = self._lin.get(id(layer))
        if spec is None:
            spec = ops.make_linear(layer.weights.detach().t(), layer.bias, None, self.dev,
                                   cin_p=ops.pad4(layer.in_channel))
            self._lin[id(layer)] = spec
            self.keep.append(spec)
        np_ = ops.pad4(spec.cout)
        if add_gemm(self.plan, a=a, a_off=a_co, lda=a_cs, M=M, wt=spec.wt[0], K=spec.cin_p, N=np_, scale=spec.scale,
                    bias=spec.bias, out=out, ldo=out.shape[-1], relu=False, cin=spec.cin, cout=spec.cout,
                    tag="gcn_gemm"):
            return
        add_conv(self.plan, x=ptr(a), x_cs=a_cs, x_co=a_co, B=1, Hi=1, Wi=M, cin_p=spec.cin_p, Hg=1, Wg=M, in_s=1,
                 taps=[(0, 0)], wt=ptr(spec.wt[0]), N=np_, n_store=np_, scale=ptr(spec.scale), bias=ptr(spec.bias),
                 out=ptr(out), out_cs=out.shape[-1], out_co=0, Ho=1, Wo=M, cin=spec.cin, cout=spec.cout,
                 tag="gcn_gemm")


def _off(t, floats):
    return ptr(t) if floats == 0 else type(ptr(t))(t.data_ptr() + 4 * floats)


def _level0_branch(e: _Emit, fu: FusionNetLite, bi: int, br: str, N: int, idx0, v, v_bs, v_st, F0, Y1b, feat1, cy: int):
    """Level-0 branch `br` up to its pool (fusion.py:183-196): conv_0 (Conv_surface + ReLU) and
    conv_1 (Conv_layer + BN1d + ReLU, its GEMM and gather-conv in crop chunks of cy) on the
    branch's vertices v (rows of stride v_st floats)."""
    B = e.B
    c0 = getattr(fu, f"conv_0_{br}")
    e.gcn(idx0, N, fu.neighbor_num, v, v_bs, 3, _dn(c0.directions, e.dev), 128, None, None, True,
          _off(F0, 128 * bi), N * 384, 384, v_st=v_st)
    c1 = getattr(fu, f"conv_1_{br}")
    dn1, bn1 = _dn(c1.directions, e.dev), _bn1d(getattr(fu, f"bn1_{br}"), e.dev)
    for b0 in range(0, B, cy):
        nb = min(cy, B - b0)
        e.gemm(F0[b0:b0 + nb], 384, 128 * bi, nb * N, c1, Y1b)
        vb = type(v)(v.value + 4 * b0 * v_bs)
        e.gcn(idx0[b0:b0 + nb], N, fu.neighbor_num, vb, v_bs, 3, dn1, 128, Y1b, bn1, True,
              _off(feat1[b0:], 128 * bi), N * 384, 384, Bc=nb, v_st=v_st)


def emit_fusion_cloud_part(fu: FusionNetLite, plan: Plan, B: int, N: int, cloud: torch.Tensor) -> dict:
    """The fusion work that reads only the input cloud ([B, N, 3]): the level-0 kNN idx0
    (fusion.py:175) and the v branch's conv_0 / conv_1 (fusion.py:183-189, whose vertices are the
    cloud). KRRNPlan emits it at the start of the forward on a side stream, beside the HRNet
    phase that leaves most of the chip idle; build_fusion_plan(early=...) then skips it. Same
    launches on the same values (the cloud is p9's first three channels): bit-identical."""
    k0 = fu.neighbor_num
    keep: list = []
    e = _Emit(fu, plan, B, keep)
    cy = B if not FUSION_CHUNK or FUSION_CHUNK >= B else FUSION_CHUNK
    idx0 = plan.buf((B, N, k0), torch.int32)
    F0 = plan.buf((B, N, 384))
    feat1 = plan.buf((B, N, 384))
    Y1v = plan.buf((cy * N, (fu.support_num + 1) * 128))
    e.knn(ptr(cloud), N * 3, 3, N, ptr(None), ptr(cloud), N * 3, 3, N, 3, k0, 1, 0, idx0)
    _level0_branch(e, fu, 0, "v", N, idx0, ptr(cloud), N * 3, 3, F0, Y1v, feat1, cy)
    plan.buffers.append(keep)
    return dict(idx0=idx0, F0=F0, feat1=feat1, Y1v=Y1v)


def build_fusion_plan(fu: FusionNetLite, plan: Plan, B: int, N: int, p9: torch.Tensor, perms: Dict[str, torch.Tensor],
                      hooks: Optional[Dict[str, List[Callable[[dict], None]]]] = None, materialize: bool = True,
                      early: Optional[dict] = None):
    """Emit FusionNetLite.forward for P9 = [cloud | xyz_emb | nml_emb] ([B, N, 9] f32).

    perms: int32 device buffers 'v', 'x', 'n' ([N1] each, permutations of N), 'p1' ([N1]),
    'p2' ([N2], permutation of N1), filled before the plan runs. Returns the [B, N, 1280] buffer.
    hooks: optional callables run at named points of the emission ('level1' = after the level-1
    branch join, 'level2' = after the level-2 kNN), each given the level buffers complete at that
    point (feat1, feat2), e.g. to fork independent work onto a side stream where the fusion
    leaves the chip underused. materialize=False skips writing the 1280-wide concat (returns None
    for it): its only consumer, TBase conv1, reads the level rows by linearity.
    early: emit_fusion_cloud_part's buffers when that part was emitted already (joined before this).
    """
    hooks = hooks or {}
    dev = plan.device
    S = fu.support_num
    k0 = fu.neighbor_num
    N1, N2, k1, k2 = level_sizes(N, k0)
    if k1 < 1 or k2 < 1:
        raise ValueError(f"num_points={N} too small for the 3-level GCN (needs N/16 >= 8)")
    keep = []
    i32 = torch.int32
    idx0 = early["idx0"] if early else plan.buf((B, N, k0), i32)
    F0 = early["F0"] if early else plan.buf((B, N, 384))
    # one GEMM-output buffer per branch: the three branches run on their own plan streams. With
    # FUSION_CHUNK = c the level-0 GEMM and its gather-conv run in crop chunks of c through a
    # c-crop buffer per branch (crops are independent: a point's neighbours are in its own crop),
    # so Y is written and re-read while it sits in the Infinity Cache instead of one 262 MB HBM
    # round trip per branch; the buffer is reused by every chunk
    cy = B if not FUSION_CHUNK or FUSION_CHUNK >= B else FUSION_CHUNK
    Y1 = [early["Y1v"] if early and i == 0 else plan.buf((cy * N, (S + 1) * 128)) for i in range(3)]
    feat1 = early["feat1"] if early else plan.buf((B, N, 384))
    nb4 = {br: plan.buf((B, N1, 4), i32) for br in ("v", "x", "n")}
    V1 = plan.buf((B, N1, 9))
    FP1 = plan.buf((B, N1, 384))
    PV1 = plan.buf((B, N1, 9))
    idx1 = plan.buf((B, N1, k1), i32)
    Y2 = [plan.buf((B * N1, (S + 1) * 128)) for _ in range(3)]
    feat2 = plan.buf((B, N1, 384))
    nb4b = plan.buf((B, N2, 4), i32)
    FP2 = plan.buf((B, N2, 384))
    PV2 = plan.buf((B, N2, 9))
    idx2 = plan.buf((B, N2, k2), i32)
    Y4 = plan.buf((B * N2, (S + 1) * 512))
    fm4 = plan.buf((B, N2, 512))
    Y5 = plan.buf((B * N2, (S + 1) * 512))
    fm5 = plan.buf((B, N2, 512))
    nn1 = plan.buf((B, N), i32)
    nn2 = plan.buf((B, N), i32)
    feat = plan.buf((B, N, 1280)) if materialize else None

    e = _Emit(fu, plan, B, keep)
    knn, gcn, gemm, off = e.knn, e.gcn, e.gemm, _off

    # level 0: idx0 = kNN(cloud, 10) (fusion.py:175)
    # level 0: idx0 = kNN(cloud, 10) (fusion.py:175); then the v / x / n branches (conv_0,
    # conv_1 + BN + ReLU, pool_1_*) are independent until the concat: branch bi on stream bi
    if not early:
        knn(off(p9, 0), N * 9, 9, N, ptr(None), off(p9, 0), N * 9, 9, N, 3, k0, 1, 0, idx0)
    plan.fork([1, 2])
    for bi, br in enumerate(("v", "x", "n")):
        with plan.on_stream(bi):
            if not (early and bi == 0):
                _level0_branch(e, fu, bi, br, N, idx0, off(p9, 3 * bi), N * 9, 9, F0, Y1[bi], feat1, cy)
            # pools (fusion.py:197-202): kNN(4) at the sampled rows, max, vertex gather
            perm = perms[br]
            knn(off(p9, 3 * bi), N * 9, 9, N1, ptr(perm), off(p9, 3 * bi), N * 9, 9, N, 3, 4, 1, 0, nb4[br])
            plan.add("krrn_pool_max_f32", ptr(nb4[br]), N1, 4, off(feat1, 128 * bi), N * 384, 384, 128,
                     off(FP1, 128 * bi), N1 * 384, 384, B)
            plan.add("krrn_gather_rows_f32", ptr(perm), 0, 0, N1, off(p9, 3 * bi), N * 9, 9, off(V1, 3 * bi),
                     N1 * 9, 9, 3, B)
    plan.add("krrn_gather_rows_f32", ptr(perms["p1"]), 0, 0, N1, off(p9, 0), N * 9, 9, off(PV1, 0), N1 * 9, 9, 9, B)
    plan.join([1, 2])
    # level 1 (fusion.py:205-216)
    knn(off(V1, 0), N1 * 9, 9, N1, ptr(None), off(V1, 0), N1 * 9, 9, N1, 3, k1, 1, 0, idx1)
    plan.fork([1, 2, 3])
    with plan.on_stream(3):  # nearest-index to pool_1 (fusion.py:231) only needs PV1
        knn(off(p9, 0), N * 9, 9, N, ptr(None), off(PV1, 0), N1 * 9, 9, N1, 3, 1, 0, 1, nn1)
    for bi, br in enumerate(("v", "x", "n")):
        with plan.on_stream(bi):
            c2 = getattr(fu, f"conv_2_{br}")
            gemm(FP1, 384, 128 * bi, B * N1, c2, Y2[bi])
            gcn(idx1, N1, k1, off(V1, 3 * bi), N1 * 9, 3, _dn(c2.directions, dev), 128, Y2[bi],
                _bn1d(getattr(fu, f"bn2_{br}"), dev), True, off(feat2, 128 * bi), N1 * 384, 384)
    plan.join([1, 2])
    for h in hooks.get("level1", []):
        h(dict(feat1=feat1, feat2=feat2))
    # pool_2 (fusion.py:219): kNN on pool_1[..., :3] at the sampled rows
    knn(off(PV1, 0), N1 * 9, 9, N2, ptr(perms["p2"]), off(PV1, 0), N1 * 9, 9, N1, 3, 4, 1, 0, nb4b)
    plan.add("krrn_pool_max_f32", ptr(nb4b), N2, 4, off(feat2, 0), N1 * 384, 384, 384, off(FP2, 0), N2 * 384, 384, B)
    plan.add("krrn_gather_rows_f32", ptr(perms["p2"]), 0, 0, N2, off(PV1, 0), N1 * 9, 9, off(PV2, 0), N2 * 9, 9, 9, B)
    # level 2 (fusion.py:223-229): 9-D kNN, Conv_fuse_layer x2, no activation
    knn(off(PV2, 0), N2 * 9, 9, N2, ptr(None), off(PV2, 0), N2 * 9, 9, N2, 9, k2, 1, 0, idx2)
    for h in hooks.get("level2", []):
        h(dict(feat1=feat1, feat2=feat2))
    plan.fork([3])
    with plan.on_stream(3):  # nearest-index to pool_2 (fusion.py:232)
        knn(off(p9, 0), N * 9, 9, N, ptr(None), off(PV2, 0), N2 * 9, 9, N2, 3, 1, 0, 1, nn2)
    gemm(FP2, 384, 0, B * N2, fu.conv_4, Y4)
    gcn(idx2, N2, k2, off(PV2, 0), N2 * 9, 9, _dn(fu.conv_4.directions, dev), 512, Y4, None, False,
        off(fm4, 0), N2 * 512, 512)
    gemm(fm4, 512, 0, B * N2, fu.conv_5, Y5)
    gcn(idx2, N2, k2, off(PV2, 0), N2 * 9, 9, _dn(fu.conv_5.directions, dev), 512, Y5, None, False,
        off(fm5, 0), N2 * 512, 512)
    # the 1280-wide concat (fusion.py:234-238). TBase consumes it by linearity from the level rows
    # (posenet.build_tbase_plan), so the materialised concat (the module's output, kept for
    # inspection) is written on side stream FEAT_SID, off the critical path; the caller joins it.
    plan.join([3])
    if materialize:
        plan.fork([FEAT_SID])
        with plan.on_stream(FEAT_SID):
            plan.add("krrn_gather_rows_f32", ptr(nn2), 0, N, N, off(fm5, 0), N2 * 512, 512, off(feat, 0), N * 1280,
                     1280, 512, B)
            plan.add("krrn_gather_rows_f32", ptr(nn1), 0, N, N, off(feat1, 0), N * 384, 384, off(feat, 512),
                     N * 1280, 1280, 384, B)
            plan.add("krrn_gather_rows_f32", ptr(nn1), 0, N, N, off(feat2, 0), N1 * 384, 384, off(feat, 896),
                     N * 1280, 1280, 384, B)
    plan.buffers.append(keep)
    return feat, dict(pool_v=nb4["v"], pool_x=nb4["x"], pool_n=nb4["n"], pool2=nb4b, idx0=idx0, idx1=idx1, idx2=idx2, nn1=nn1, nn2=nn2, feat1=feat1, feat2=feat2, fm5=fm5,
                      F0=F0, V1=V1, PV1=PV1, PV2=PV2, FP1=FP1, FP2=FP2, fm4=fm4, Y1=Y1, Y2=Y2, Y4=Y4, Y5=Y5)
