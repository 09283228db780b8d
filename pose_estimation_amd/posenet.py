"""Translation head of KRRN (lib/network/pose/posenet.py:51-96), MI355X execution.

TBase = Conv1d(1280 + C -> 1024) + BN + ReLU -> (-> 256) + BN + ReLU -> (-> 256) + BN + ReLU
        -> Dropout (eval: identity) -> Conv1d(-> OUT_T); t_res = [:, 0:3]
and KRRN.forward's pred_t = mean_N(p_emb + t_res) (krrn.py:153).

Execution: the one-hot class channels of the concat (krrn.py:132-138) contribute exactly the
column W1[:, 1280 + cls] to conv1, so they become a per-crop bias (one gather launch) instead
of C extra input channels; conv1 runs by linearity on the fusion's level rows (see
build_tbase_plan); conv1..conv3 are f32-MFMA GEMMs with BN folded into the epilogue;
conv4 + the mean over points is one reduction launch per crop.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import knobs, ops
from .runtime import Late, Plan, add_conv, add_gemm, ptr


# conv2 gathers h1 = ReLU(P1[nn1] + P2[nn2]) inside its operand staging (krrn_gemm_x3_gather_f32)
# instead of a separate gather-add launch writing the 262 MB h1 (KRRN_TBASE_GATHER=0: the old form)
TBASE_GATHER = knobs.flag("KRRN_TBASE_GATHER")


class TBase(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.f = cfg.Module.POSENet.INC_R + cfg.Module.NUM_CLS
        self.k = cfg.Module.POSENet.OUT_T
        self.conv1 = nn.Conv1d(self.f, 1024, 1)
        self.conv2 = nn.Conv1d(1024, 256, 1)
        self.conv3 = nn.Conv1d(256, 256, 1)
        self.conv4 = nn.Conv1d(256, self.k, 1)
        self.drop1 = nn.Dropout(0.2)
        self.bn1 = nn.BatchNorm1d(1024)
        self.bn2 = nn.BatchNorm1d(256)
        self.bn3 = nn.BatchNorm1d(256)


class PoseNet(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.t_net = TBase(cfg)


def _conv1_fold(tb: TBase, inc_r: int, num_cls: int, dev):
    """conv1 + bn1 folded: (W1 [1024, inc_r + C], spec1 with the BN scale / bias, colv [C, 1024] =
    the one-hot columns pre-multiplied by the BN scale)."""
    w1 = tb.conv1.weight.detach()[:, :, 0]
    spec1 = ops.make_linear(w1[:, :inc_r], tb.conv1.bias, tb.bn1, dev)
    np1 = ops.pad4(1024)
    colv = torch.zeros(num_cls, np1, device=dev)
    colv[:, :1024] = (spec1.scale[:1024, None] * w1[:, inc_r:inc_r + num_cls].to(dev).float()).t()
    return w1, spec1, colv


def emit_tbase_level1(tb: TBase, plan: Plan, B: int, N: int, N1: int, feat1: torch.Tensor,
                      feat2: torch.Tensor, cls_key: str = "cls", inc_r: int = 1280, num_cls: int = 1) -> dict:
    """The part of TBase conv1 (by linearity, see build_tbase_plan) that needs only the level-0 /
    level-1 features: P1 = feat1[:N1] W1[:, 512:896]^T + feat2 W1[:, 896:1280]^T, on the plan's
    current stream. Emitted from the fusion's 'level1' hook, it runs beside the level-2 GCN chain.
    With TBASE_GATHER the BN scale is folded into those weights and the BN shift + conv1 bias + the
    crop's one-hot column are added here, so conv2 only has to gather, add and ReLU (fused into its
    operand staging, krrn_gemm_x3_gather_f32)."""
    dev = plan.device
    np1 = ops.pad4(1024)
    if TBASE_GATHER:
        w1, spec1, colv = _conv1_fold(tb, inc_r, num_cls, dev)
        wb = ops.make_linear(w1[:, 512:896], None, None, dev)
        wc = ops.make_linear(w1[:, 896:1280], None, None, dev)
        b2 = plan.buf((B, np1))
        plan.add("krrn_gather_rows_f32", Late(cls_key), 1, 1, 1, ptr(colv), 0, np1, ptr(b2), np1, np1, np1, B)
        Q = plan.buf((B * N1, np1))
        P1 = plan.buf((B * N1, np1))
        # Q = s (feat2 Wc) + shift + b2[crop] (the crop's row of b2 broadcast: ldr = 0, one row per group)
        ok = add_gemm(plan, a=feat2, a_off=0, lda=384, M=N1, wt=wc.wt[0], K=wc.cin_p, N=np1, scale=spec1.scale,
                      bias=spec1.bias, out=Q, ldo=np1, relu=False, res=b2, ldr=0, batch=B, a_grp=N1 * 384,
                      o_grp=N1 * np1, r_grp=np1, cin=wc.cin, cout=wc.cout, tag="tbase_gemm", require_x3=True) and \
            add_gemm(plan, a=feat1, a_off=0, lda=384, M=N1, wt=wb.wt[0], K=wb.cin_p, N=np1, scale=spec1.scale,
                     bias=None, out=P1, ldo=np1, relu=False, res=Q, ldr=np1, batch=B, a_grp=N * 384,
                     o_grp=N1 * np1, r_grp=N1 * np1, cin=wb.cin, cout=wb.cout, tag="tbase_gemm", require_x3=True)
        if not ok:
            raise RuntimeError("TBase gathered conv2 needs the split-bf16 GEMM (KRRN_GEMM_X3=1)")
        plan.buffers.append([wb, wc, spec1, colv])
        return dict(P1=P1, Q=Q, b2=b2, folded=True)
    w1 = tb.conv1.weight.detach()[:, :, 0]
    wb = ops.make_linear(w1[:, 512:896], None, None, dev)
    wc = ops.make_linear(w1[:, 896:1280], None, None, dev)
    Q = plan.buf((B * N1, np1))
    P1 = plan.buf((B * N1, np1))
    if add_gemm(plan, a=feat2, a_off=0, lda=384, M=B * N1, wt=wc.wt[0], K=wc.cin_p, N=np1, scale=wc.scale,
                bias=wc.bias, out=Q, ldo=np1, relu=False, cin=wc.cin, cout=wc.cout, tag="tbase_gemm") and \
            add_gemm(plan, a=feat1, a_off=0, lda=384, M=N1, wt=wb.wt[0], K=wb.cin_p, N=np1, scale=wb.scale,
                     bias=wb.bias, out=P1, ldo=np1, relu=False, res=Q, ldr=np1, batch=B, a_grp=N * 384,
                     o_grp=N1 * np1, r_grp=N1 * np1, cin=wb.cin, cout=wb.cout, tag="tbase_gemm"):
        plan.buffers.append([wb, wc])
        return dict(P1=P1, Q=Q)
    add_conv(plan, x=ptr(feat2), x_cs=384, x_co=0, B=1, Hi=1, Wi=B * N1, cin_p=wc.cin_p, Hg=1, Wg=B * N1, in_s=1,
             taps=[(0, 0)], wt=ptr(wc.wt[0]), N=np1, n_store=np1, scale=ptr(wc.scale), bias=ptr(wc.bias),
             out=ptr(Q), out_cs=np1, out_co=0, Ho=1, Wo=B * N1, relu=False, cin=wc.cin, cout=wc.cout,
             tag="tbase_gemm")
    # feat1 rows 0..N1-1 of every crop (grid B x N1 over images of N points), + Q
    add_conv(plan, x=ptr(feat1), x_cs=384, x_co=0, B=B, Hi=1, Wi=N, cin_p=wb.cin_p, Hg=1, Wg=N1,
             in_s=1, taps=[(0, 0)], wt=ptr(wb.wt[0]), N=np1, n_store=np1, scale=ptr(wb.scale), bias=ptr(wb.bias),
             res=ptr(Q), res_cs=np1, res_co=0, out=ptr(P1), out_cs=np1, out_co=0, Ho=1, Wo=N1, relu=False,
             cin=wb.cin, cout=wb.cout, tag="tbase_gemm")
    plan.buffers.append([wb, wc])
    return dict(P1=P1, Q=Q)


def build_tbase_plan(tb: TBase, plan: Plan, B: int, N: int, feat: torch.Tensor, cls_key: str, cloud_key: str,
                     inc_r: int, num_cls: int, levels=None, pre: Optional[dict] = None, pre_sid: int = 0):
    """Emit TBase + pred_t. `feat` is [B, N, inc_r]; cls ([B, 1] int64) and cloud ([B, N, 3])
    are late-bound env tensors. Returns the [B, 3] pred_t buffer.

    With `levels` (the fusion's level rows fm5 [B, N2, 512], feat1 [B, N, 384], feat2 [B, N1, 384]
    and the nearest indices nn1 / nn2 that build the concat, fusion.py:230-238), conv1 runs by
    linearity on the level rows instead of the N gathered rows: P2 = fm5 W1[:, :512]^T (N2 rows),
    P1 = feat1[:N1] W1[:, 512:896]^T + feat2 W1[:, 896:1280]^T (N1 rows; the reference indexes
    feat_1 with nearest_pool_1, so only its first N1 rows are ever read), then one gather-add
    launch applies BN + one-hot column + ReLU per point. 29 instead of 168 GFLOP at config 2.
    `pre`: P1 already emitted by emit_tbase_level1 on stream `pre_sid` (joined here before use)."""
    dev = plan.device
    # one-hot columns, pre-multiplied by the folded BN scale: colv[c] = scale * W1[:, inc_r + c]
    w1, spec1, colv = _conv1_fold(tb, inc_r, num_cls, dev)
    np1 = ops.pad4(1024)
    spec2 = ops.make_linear(tb.conv2.weight, tb.conv2.bias, tb.bn2, dev)
    spec3 = ops.make_linear(tb.conv3.weight, tb.conv3.bias, tb.bn3, dev)
    w4 = tb.conv4.weight.detach()[:3, :, 0].float().contiguous().to(dev)
    b4 = tb.conv4.bias.detach()[:3].float().contiguous().to(dev)
    gathered = levels is not None and TBASE_GATHER
    h1 = None if gathered else plan.buf((B * N, 1024))
    h2 = plan.buf((B * N, 256))
    h3 = plan.buf((B * N, 256))
    pred_t = plan.buf((B, 3))
    M = B * N
    keep = [spec1, spec2, spec3, colv, w4, b4]
    if not gathered:
        b2 = plan.buf((B, np1))
        plan.add("krrn_gather_rows_f32", Late(cls_key), 1, 1, 1, ptr(colv), 0, np1, ptr(b2), np1, np1, np1, B)

    def gemm(a, K, spec, out, bias2=None, rows=M, relu=True):
        np_ = ops.pad4(spec.cout)
        if bias2 is None and add_gemm(plan, a=a, a_off=0, lda=K, M=rows, wt=spec.wt[0], K=spec.cin_p, N=np_,
                                      scale=spec.scale, bias=spec.bias, out=out, ldo=out.shape[-1], relu=relu,
                                      cin=spec.cin, cout=spec.cout, tag="tbase_gemm"):
            return
        add_conv(plan, x=ptr(a), x_cs=K, x_co=0, B=1, Hi=1, Wi=rows, cin_p=spec.cin_p, Hg=1, Wg=rows, in_s=1,
                 taps=[(0, 0)], wt=ptr(spec.wt[0]), N=np_, n_store=np_, scale=ptr(spec.scale), bias=ptr(spec.bias),
                 bias2=ptr(bias2) if bias2 is not None else None, b2_div=N, out=ptr(out), out_cs=out.shape[-1],
                 out_co=0, Ho=1, Wo=rows, relu=relu, cin=spec.cin, cout=spec.cout, tag="tbase_gemm")

    if levels is None:
        gemm(feat, inc_r, spec1, h1, bias2=b2)
    else:
        N1, N2 = levels["N1"], levels["N2"]
        wa = ops.make_linear(w1[:, 0:512], None, None, dev)
        keep += [wa]
        P2 = plan.buf((B * N2, np1))
        if gathered:  # BN scale folded into W1's columns, as for P1 (emit_tbase_level1)
            if not add_gemm(plan, a=levels["fm5"], a_off=0, lda=512, M=B * N2, wt=wa.wt[0], K=wa.cin_p, N=np1,
                            scale=spec1.scale, bias=None, out=P2, ldo=np1, relu=False, cin=wa.cin, cout=wa.cout,
                            tag="tbase_gemm", require_x3=True):
                raise RuntimeError("TBase gathered conv2 needs the split-bf16 GEMM (KRRN_GEMM_X3=1)")
        else:
            gemm(levels["fm5"], 512, wa, P2, rows=B * N2, relu=False)
        if pre is None:
            pre = emit_tbase_level1(tb, plan, B, N, N1, levels["feat1"], levels["feat2"], cls_key=cls_key,
                                    inc_r=inc_r, num_cls=num_cls)
        else:
            plan.join([pre_sid])
        P1 = pre["P1"]
        if gathered:
            # conv2 with h1 = ReLU(P1[nn1] + P2[nn2]) built in its operand staging (never in HBM)
            w2 = tb.conv2.weight.detach()[:, :, 0].to(dev).float() * spec2.scale[:256].reshape(256, 1)
            w3 = ops.gemm_weights_x3(w2.contiguous())
            keep += [w3]
            plan.add("krrn_gemm_x3_gather_f32", ptr(levels["nn1"]), ptr(P1), N1 * np1, np1, ptr(levels["nn2"]),
                     ptr(P2), N2 * np1, np1, N, B, 1024, 256, ptr(w3), ptr(spec2.bias), ptr(h2), 256, 1,
                     meta=dict(kernel="gemm_x3", flops=2.0 * 1024 * 256 * M, tag="tbase_gemm", M=M, N=256, K=1024,
                               splits=1, mfma_flops=2.0 * M * 256 * 1024 * 6 / 16,
                               mfma_bf16_flops=2.0 * M * 256 * 1024 * 6))
        else:
            plan.add("krrn_gather2_add_f32", ptr(levels["nn2"]), ptr(P2), N2 * np1, np1, ptr(levels["nn1"]),
                     ptr(P1), N1 * np1, np1, N, np1, ptr(spec1.scale), ptr(spec1.bias), ptr(b2), 1, ptr(h1),
                     N * 1024, 1024, B)
    if not gathered:
        gemm(h1, 1024, spec2, h2)
    gemm(h2, 256, spec3, h3)
    plan.add("krrn_tbase_tail_f32", ptr(h3), B, N, 256, ptr(w4), ptr(b4), Late(cloud_key), ptr(pred_t), ptr(None))
    plan.buffers.append(keep)
    return pred_t, dict(h1=h1, h2=h2, h3=h3)
