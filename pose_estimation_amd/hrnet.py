"""HRNet backbone of KRRN (lib/network/hrnet/myhrnet.py:28-527), MI355X execution.

The nn.Module tree below only *holds parameters*, with exactly the reference's attribute
names and nn.Sequential positions so that reference checkpoints load unchanged
(`backbone.conv1`, `backbone.layer1.0.downsample.1`, `backbone.stage3.2.fuse_layers.2.0.1.0`,
`backbone.last_layer.0.0`, `backbone.deconv_layer.1.0.conv1`, ...). The forward
is compiled by `build_hrnet_plan` into NHWC HIP launches:

  * every conv + eval-BN (+ residual add) (+ ReLU) is ONE implicit-GEMM launch
    (krrn_conv2d_f32) with BN folded into a per-channel scale/bias;
  * the multi-resolution fuse (myhrnet.py:226-250) accumulates into the output branch
    buffer: j < i chains end in a conv whose epilogue adds the running sum, j > i terms
    are a 1x1 conv at the low resolution followed by one bilinear-resize-add launch
    (align_corners=False, myhrnet.py:242-245), the last term applies the ReLU;
  * the final upsample + concat (myhrnet.py:511-516) resizes each branch straight into
    its channel slice of the concat buffer, and last_layer / deconv_layer (:518-525)
    write into channel slices so no torch.cat ever copies.
Channel counts that are not multiples of 4 (W18: 18, 36, ...) are padded to 4 in memory;
pad channels are exactly zero and the packed weights map logical -> physical channels.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import knobs, ops
from .config import load_hrnet_spec
from .ops import Act, pad4
from .runtime import add_conv_group, add_gemm, Plan, add_conv, ptr

# switches (pose_estimation_amd/knobs.py has each one's meaning)
DECONV_FOLD = knobs.flag("KRRN_DECONV_FOLD")
CONVT_S2 = knobs.flag("KRRN_CONVT_S2")
SMALL_CONV = knobs.flag("KRRN_SMALL_CONV")
GEMM_1X1 = knobs.flag("KRRN_GEMM_1X1")
FUSE_ID_FIRST = knobs.flag("KRRN_FUSE_ID_FIRST")
WINO_X3 = knobs.flag("KRRN_WINO_X3")
# a head's final 1x1 conv with <= 4 outputs (nml_final of a one-class model) fused into the split
# Winograd of the conv before it (krrn_conv3x3_wino_x3_head_f32): its 128-channel input map is never
# written or re-read
HEAD_FUSE = knobs.flag("KRRN_HEAD_FUSE")
# each HRNet fuse output waits for the branches it reads through capture edges (runtime.Edge)
# instead of the module barrier (join into stream 0 + fork)
FUSE_EDGES = knobs.flag("KRRN_FUSE_EDGES")
# the fuse-layer work that reads only branch j's output (the 1x1 convs of the j > i terms, all but
# the last stride-2 conv of the j < i chains) runs on branch j's stream right after its blocks,
# beside the other branches' tails, instead of after the join on the output's stream
FUSE_EARLY = knobs.flag("KRRN_FUSE_EARLY")
# between two modules of a stage, branch i of the next module waits only for fuse output i (the same
# stream) instead of a join of every stream followed by a fork
MODULE_STREAMS = knobs.flag("KRRN_MODULE_STREAMS")
# ... and across stage boundaries: a stage's last module keeps its outputs on their streams, and the
# next stage's transition conv for branch i runs on stream i after a wait on its source's stream
STAGE_STREAMS = knobs.flag("KRRN_STAGE_STREAMS")
# k order of the grouped transposed convs: channel chunks of this many channels outer, taps inner
# (krrn_conv_desc.k_chunk; 0 = tap-major)
CONVT_KCHUNK = 16

BN_MOMENTUM = 0.1


def conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.downsample = downsample
        self.stride = stride


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes, momentum=BN_MOMENTUM)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4, momentum=BN_MOMENTUM)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


class HighResolutionModule(nn.Module):
    def __init__(self, num_branches, blocks, num_inchannels, num_channels):
        super().__init__()
        if not (num_branches == len(blocks) == len(num_inchannels) == len(num_channels)):
            raise ValueError("HRNet stage spec: branch count mismatch")
        self.num_branches = num_branches
        self.num_inchannels = list(num_inchannels)
        branches = []
        for i in range(num_branches):
            down = None
            if self.num_inchannels[i] != num_channels[i]:
                down = nn.Sequential(nn.Conv2d(self.num_inchannels[i], num_channels[i], 1, 1, bias=False),
                                     nn.BatchNorm2d(num_channels[i], momentum=BN_MOMENTUM))
            layers = [BasicBlock(self.num_inchannels[i], num_channels[i], 1, down)]
            self.num_inchannels[i] = num_channels[i]
            for _ in range(1, blocks[i]):
                layers.append(BasicBlock(self.num_inchannels[i], num_channels[i]))
            branches.append(nn.Sequential(*layers))
        self.branches = nn.ModuleList(branches)
        self.fuse_layers = self._make_fuse_layers() if num_branches > 1 else None
        self.relu = nn.ReLU(True)

    def _make_fuse_layers(self):
        nb, ch = self.num_branches, self.num_inchannels
        fuse = []
        for i in range(nb):
            row = []
            for j in range(nb):
                if j > i:
                    row.append(nn.Sequential(nn.Conv2d(ch[j], ch[i], 1, 1, 0, bias=False),
                                             nn.BatchNorm2d(ch[i], momentum=BN_MOMENTUM)))
                elif j == i:
                    row.append(None)
                else:
                    chain = []
                    for k in range(i - j):
                        last = k == i - j - 1
                        cout = ch[i] if last else ch[j]
                        mods = [nn.Conv2d(ch[j], cout, 3, 2, 1, bias=False), nn.BatchNorm2d(cout, momentum=BN_MOMENTUM)]
                        if not last:
                            mods.append(nn.ReLU(True))
                        chain.append(nn.Sequential(*mods))
                    row.append(nn.Sequential(*chain))
            fuse.append(nn.ModuleList(row))
        return nn.ModuleList(fuse)


class HRNet(nn.Module):
    """Parameter container with the reference's module names (myhrnet.py:258-346)."""

    def __init__(self, spec, backbone_outc: int):
        super().__init__()
        self.spec = spec
        self.conv1 = nn.Conv2d(3, 64, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64, momentum=BN_MOMENTUM)
        self.conv2 = nn.Conv2d(64, 64, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(64, momentum=BN_MOMENTUM)
        self.relu = nn.ReLU(inplace=True)
        down = nn.Sequential(nn.Conv2d(64, 256, 1, 1, bias=False), nn.BatchNorm2d(256, momentum=BN_MOMENTUM))
        self.layer1 = nn.Sequential(Bottleneck(64, 64, 1, down), *[Bottleneck(256, 64) for _ in range(3)])
        pre = [256]
        self.stage_branches: List[int] = []
        for si, st in enumerate(spec.stages):
            widths = list(st.widths)
            setattr(self, f"transition{si + 1}", self._make_transition(pre, widths))
            mods = []
            inch = list(widths)
            for _ in range(st.modules):
                m = HighResolutionModule(len(widths), list(st.blocks), inch, widths)
                mods.append(m)
                inch = m.num_inchannels
            setattr(self, f"stage{si + 2}", nn.Sequential(*mods))
            pre = inch
            self.stage_branches.append(len(widths))
        L = sum(pre)
        self.last_inp_channels = L
        self.last_layer = nn.ModuleList([
            nn.Sequential(nn.Conv2d(L, L, kernel_size=(3, 3), stride=(1, 1), padding='same'),
                          nn.BatchNorm2d(L, momentum=BN_MOMENTUM), nn.ReLU(True)),
            nn.Conv2d(L, backbone_outc, kernel_size=(1, 1), stride=(1, 1), padding=0)])
        self.deconv_layer = nn.ModuleList([
            nn.Sequential(nn.ConvTranspose2d(L + backbone_outc, backbone_outc, kernel_size=(4, 4), stride=(2, 2),
                                             padding=(1, 1), bias=False),
                          nn.BatchNorm2d(backbone_outc, eps=1e-05, momentum=0.1), nn.ReLU(True)),
            nn.Sequential(BasicBlock(backbone_outc, backbone_outc))])
        self.backbone_outc = backbone_outc

    @staticmethod
    def _make_transition(pre: List[int], cur: List[int]):
        layers = []
        for i in range(len(cur)):
            if i < len(pre):
                if cur[i] != pre[i]:
                    layers.append(nn.Sequential(nn.Conv2d(pre[i], cur[i], 3, 1, 1, bias=False),
                                                nn.BatchNorm2d(cur[i]), nn.ReLU(True)))
                else:
                    layers.append(None)
            else:
                chain = []
                for j in range(i + 1 - len(pre)):
                    cin = pre[-1]
                    cout = cur[i] if j == i - len(pre) else cin
                    chain.append(nn.Sequential(nn.Conv2d(cin, cout, 3, 2, 1, bias=False), nn.BatchNorm2d(cout),
                                               nn.ReLU(True)))
                layers.append(nn.Sequential(*chain))
        return nn.ModuleList(layers)


def build_hrnet(cfg) -> HRNet:
    """build_modeifed_hrnet(config, cfg_name) equivalent (myhrnet.py:538-547)."""
    return HRNet(load_hrnet_spec(cfg.Module.BACKBONE), cfg.Module.BACKBONE_OUTC)


# ---------------------------------------------------------------------------------------
# Plan compilation
# ---------------------------------------------------------------------------------------

class _Builder:
    def __init__(self, plan: Plan, B: int):
        self.plan = plan
        self.B = B
        self.dev = plan.device
        self.specs = []  # keep folded weights alive

    def act(self, H, W, c, cs=None) -> Act:
        cs = pad4(c) if cs is None else cs
        t = self.plan.buf((self.B, H, W, cs))
        return Act(t, self.B, H, W, cs, 0, c)

    def conv(self, x: Act, conv: nn.Module, bn: Optional[nn.Module], out: Optional[Act] = None,
             res: Optional[Act] = None, relu: bool = False, cin_map=None) -> Act:
        if isinstance(conv, nn.ConvTranspose2d):
            spec = ops.make_convT(conv, bn, self.dev, cin_map=cin_map, cin_p=x.cp)
        else:
            spec = ops.make_conv(conv, bn, self.dev, cin_map=cin_map, cin_p=x.cp)
        self.specs.append(spec)
        Ho, Wo = ops.conv_out_hw(spec, x.H, x.W)
        if out is None:
            out = self.act(Ho, Wo, spec.cout)
        assert (out.H, out.W) == (Ho, Wo) and out.cp >= pad4(spec.cout)
        if (WINO_X3 and ops.wino_eligible(spec, x.B * Ho * Wo) and (Ho, Wo) == (x.H, x.W)
                and ops.wino4_eligible(spec, x, Ho, Wo)):
            U = ops.wino_weights_x3(ops.wino4_weights(conv, self.dev, cin_map=cin_map, cin_p=x.cp))
            self.specs.append(U)
            self.emit_wino4(x, spec, U, out, res, relu)
        elif ops.wino_eligible(spec, x.B * Ho * Wo) and x.cs % 2 == 0 and x.co % 2 == 0:
            U = ops.wino_weights(conv, self.dev, cin_map=cin_map, cin_p=x.cp)
            if WINO_X3:
                U = ops.wino_weights_x3(U)
            self.specs.append(U)
            self.emit_wino(x, spec, U, out, res, relu)
        elif SMALL_CONV and ops.small_conv_eligible(spec, x):
            self.emit_small(x, spec, out, res, relu)
        elif not (GEMM_1X1 and self.emit_gemm(x, spec, out, res, relu)):
            self.emit_conv(x, spec, out, res, relu)
        return out

    def conv_head(self, x: Act, conv: nn.Module, bn: Optional[nn.Module], final: nn.Conv2d, out: torch.Tensor,
                  n_store: int) -> bool:
        """relu(bn(conv(x))) -> final (1x1 + bias) into the NCHW map `out` (channels < n_store) as
        one split-Winograd launch plus a partial-sum pass (krrn_conv3x3_wino_x3_head_f32), for a final
        conv with at most 4 outputs (nml_final with one class, krrn.py:80-84, 98). False (nothing
        emitted) when it does not apply."""
        if not (HEAD_FUSE and WINO_X3 and isinstance(conv, nn.Conv2d) and tuple(final.kernel_size) == (1, 1)
                and tuple(final.stride) == (1, 1) and final.in_channels == conv.out_channels
                and n_store <= min(4, final.out_channels) and x.cs % 2 == 0 and x.co % 2 == 0):
            return False
        spec = ops.make_conv(conv, bn, self.dev, cin_p=x.cp)
        Ho, Wo = ops.conv_out_hw(spec, x.H, x.W)
        M = x.B * Ho * Wo
        if not ops.wino_eligible(spec, M) or (Ho, Wo) != (x.H, x.W):
            return False
        np_ = pad4(spec.cout)
        f4 = ops.wino4_eligible(spec, x, Ho, Wo)
        U = ops.wino_weights_x3((ops.wino4_weights if f4 else ops.wino_weights)(conv, self.dev, cin_p=x.cp))
        w1 = torch.zeros(4, np_, device=self.dev)
        w1[:final.out_channels, :spec.cout] = final.weight.detach().reshape(final.out_channels, -1).float().to(self.dev)
        b1 = None
        if final.bias is not None:
            b1 = torch.zeros(4, device=self.dev)
            b1[:final.out_channels] = final.bias.detach().float().to(self.dev)
        self.specs += [spec, U, w1] + ([b1] if b1 is not None else [])
        part = self.plan.scratch(((np_ + 63) // 64) * M * 4)
        if f4:
            pipe = 2.0 * 36 * spec.cin_p * np_ * x.B * ((Ho + 3) // 4) * ((Wo + 3) // 4)
        else:
            pipe = 2.0 * 16 * spec.cin_p * np_ * x.B * ((Ho + 1) // 2) * ((Wo + 1) // 2)
        meta = dict(kernel="wino_f43_x3_head" if f4 else "wino_f23_x3_head", tag="conv_wino_head", M=M, N=np_,
                    K=spec.cin_p * 9, flops=2.0 * spec.cin * spec.cout * 9 * M + 2.0 * spec.cout * n_store * M,
                    mfma_flops=pipe * 6 / 16, mfma_bf16_flops=pipe * 6)
        self.plan.add("krrn_conv3x3_wino4_x3_head_f32" if f4 else "krrn_conv3x3_wino_x3_head_f32", ptr(x.t), x.cs,
                      x.co, x.B, x.H, x.W, spec.cin_p, ptr(U), np_,
                      ptr(spec.scale), ptr(spec.bias), ptr(None), 0, 0, 1, ptr(w1), ptr(b1), n_store, ptr(part),
                      ptr(out), out.shape[1], meta=meta)
        return True

    def upsample2(self, x: Act) -> Act:
        """UpsamplingBilinear2d(scale 2)(x) (krrn.py:56, 78; align_corners=True) materialised for the
        conv after it. Blending the upsample into the split Winograd's input staging instead was
        measured slower and removed."""
        up = self.act(2 * x.H, 2 * x.W, x.c)
        self.resize(x, up, align=True)
        return up

    def emit_gemm(self, x: Act, spec, out: Act, res: Optional[Act], relu: bool) -> bool:
        """A wide 1x1 / stride-1 conv (layer1's Bottleneck projections, myhrnet.py:66-103) is a plain
        GEMM over the NHWC rows through add_gemm's own kernels (BN folded, residual + ReLU epilogue).
        False (nothing emitted) when none fits -- layer1's 256 -> 64 projections (K = 256, N = 64):
        they then run on the split-bf16 implicit GEMM (emit_conv), not on hipBLASLt."""
        if not (spec.kind == "conv" and spec.ksize == 1 and spec.stride == 1 and out.co == 0
                and (res is None or res.co == 0)):
            return False
        np_ = pad4(spec.cout)
        return add_gemm(self.plan, a=x.t, a_off=x.co, lda=x.cs, M=x.B * x.H * x.W, wt=spec.wt[0], K=spec.cin_p,
                        N=np_, scale=spec.scale, bias=spec.bias, out=out.t, ldo=out.cs, relu=relu,
                        res=res.t if res is not None else None, ldr=res.cs if res is not None else 0,
                        cin=spec.cin, cout=spec.cout, tag="conv1x1_gemm", blas_ok=False)

    @staticmethod
    def small_problem(x: Act, spec, out: Act, res: Optional[Act], relu: bool) -> dict:
        """krrn_conv_small_f32's arguments (SmallDesc fields) plus the breakdown's FLOP counts."""
        np_ = pad4(spec.cout)
        M = x.B * out.H * out.W
        taps = spec.ksize * spec.ksize
        ntiles = (np_ + 15) // 16
        nw, ks = ops.small_conv_config(M, ntiles, spec.cin_p)
        return dict(x=ptr(x.t), in_cs=x.cs, in_co=x.co, B=x.B, H=x.H, W=x.W, cin=spec.cin_p, wt=ptr(spec.wt[0]),
                    N=np_, n_store=np_, scale=ptr(spec.scale), bias=ptr(spec.bias),
                    res=ptr(res.t) if res is not None else ptr(None), res_cs=res.cs if res is not None else 0,
                    res_co=res.co if res is not None else 0, out=ptr(out.t), out_cs=out.cs, out_co=out.co,
                    relu=int(relu), ksize=spec.ksize, stride=spec.stride, nw=nw, ks=ks, M=M,
                    flops=2.0 * spec.cin * spec.cout * taps * M,
                    mfma_flops=2.0 * 16 * ((taps * spec.cin_p // 4 + 3) // 4) * 16 * ntiles * M)

    def emit_small(self, x: Act, spec, out: Act, res: Optional[Act], relu: bool, tag: str = "conv"):
        p = self.small_problem(x, spec, out, res, relu)
        self.plan.add("krrn_conv_small_f32", p["x"], p["in_cs"], p["in_co"], p["B"], p["H"], p["W"], p["cin"], p["wt"],
                      p["N"], p["n_store"], p["scale"], p["bias"], p["res"], p["res_cs"], p["res_co"], p["out"],
                      p["out_cs"], p["out_co"], p["relu"], p["ksize"], p["stride"], p["nw"], p["ks"],
                      meta=dict(kernel=f"conv_small<{p['nw']},{p['ks']}>", flops=p["flops"], tag=tag, M=p["M"], N=p["N"],
                                K=spec.cin_p * spec.ksize ** 2, splits=1, mfma_flops=p["mfma_flops"]))

    def emit_wino(self, x: Act, spec, U: torch.Tensor, out: Act, res: Optional[Act], relu: bool,
                  tag: str = "conv"):
        """Fused Winograd F(2x2,3x3): on the bf16 matrix cores with split operands (U = the
        wino_weights_x3 planes) or on the f32 ones (U f32)."""
        np_ = pad4(spec.cout)
        M = x.B * out.H * out.W
        x3 = U.dtype == torch.bfloat16
        tiles = x.B * ((out.H + 1) // 2) * ((out.W + 1) // 2)
        # matrix-pipe FLOPs: f32 MFMA 2 per (component, tile, channel in, channel out); the split
        # kernel issues 6 bf16 term products each (12 FLOPs) at 16x the f32 rate, counted here in
        # f32-pipe time (/ 16) so all_conv's pipe fraction stays one scale
        pipe = 2.0 * 16 * spec.cin_p * np_ * tiles
        meta = dict(kernel="wino_f23_x3" if x3 else "wino_f23<32,32,16>", flops=2.0 * spec.cin * spec.cout * 9 * M,
                    tag=tag + "_wino", M=M, N=np_, K=spec.cin_p * 9, mfma_flops=pipe * 6 / 16 if x3 else pipe)
        if x3:
            meta["mfma_bf16_flops"] = pipe * 6
        self.plan.add("krrn_conv3x3_wino_x3_f32" if x3 else "krrn_conv3x3_wino_f32", ptr(x.t), x.cs, x.co, x.B, x.H,
                      x.W, spec.cin_p, ptr(U), np_, np_, ptr(spec.scale), ptr(spec.bias),
                      ptr(res.t) if res is not None else ptr(None), res.cs if res is not None else 0,
                      res.co if res is not None else 0, ptr(out.t), out.cs, out.co, int(relu), meta=meta)

    def emit_wino4(self, x: Act, spec, U: torch.Tensor, out: Act, res: Optional[Act], relu: bool,
                   tag: str = "conv"):
        """Fused Winograd F(4x4,3x3) on split-bf16 operands (krrn_conv3x3_wino4_x3_f32; U = the
        wino_weights_x3 planes of wino4_weights)."""
        np_ = pad4(spec.cout)
        M = x.B * out.H * out.W
        tiles = x.B * ((out.H + 3) // 4) * ((out.W + 3) // 4)
        pipe = 2.0 * 36 * spec.cin_p * np_ * tiles  # f32-equivalent component products (see emit_wino)
        meta = dict(kernel="wino_f43_x3", flops=2.0 * spec.cin * spec.cout * 9 * M, tag=tag + "_wino", M=M, N=np_,
                    K=spec.cin_p * 9, mfma_flops=pipe * 6 / 16, mfma_bf16_flops=pipe * 6)
        self.plan.add("krrn_conv3x3_wino4_x3_f32", ptr(x.t), x.cs, x.co, x.B, x.H, x.W, spec.cin_p, ptr(U), np_, np_,
                      ptr(spec.scale), ptr(spec.bias), ptr(res.t) if res is not None else ptr(None),
                      res.cs if res is not None else 0, res.co if res is not None else 0, ptr(out.t), out.cs,
                      out.co, int(relu), meta=meta)

    def emit_convT_s2(self, x: Act, spec, out: Act, relu: bool, tag: str = "conv"):
        """A stride-2 transposed conv with 128 outputs (the deconv, myhrnet.py:314-326; XYZNet's first
        layer, krrn.py:47-49) as ONE krrn_convT_s2_x3_f32 launch: all four parity classes of a 4 x 32
        input-grid region per block, the input staged and split once per 8-channel chunk."""
        U3, table = ops.convT_weights_x3(spec)
        self.specs.append(U3)
        taps = sum(len(t) for t in spec.taps)
        grid = x.B * (-(-x.H // 4) * 4) * (-(-x.W // 32) * 32)  # the blocks' padded input grid
        issued = 2.0 * grid * 128 * spec.cin_p * max(len(t) for t in spec.taps) * 4  # the busiest class sets the pace
        meta = dict(kernel="convt_s2_x3", flops=2.0 * spec.cin * spec.cout * taps * x.B * x.H * x.W,
                    tag=tag + "_convT", M=x.B * x.H * x.W * 4, N=128, K=spec.cin_p * taps,
                    mfma_flops=issued * 6 / 16, mfma_bf16_flops=issued * 6)
        self.plan.add("krrn_convT_s2_x3_f32", ptr(x.t), x.cs, x.co, x.B, x.H, x.W, spec.cin_p, table, ptr(U3), 128,
                      ptr(spec.scale), ptr(spec.bias), int(relu), ptr(out.t), out.cs, out.co, out.H, out.W, meta=meta)

    def emit_conv(self, x: Act, spec, out: Act, res: Optional[Act], relu: bool, tag: str = "conv"):
        np_ = pad4(spec.cout)
        if CONVT_S2 and ops.convT_s2_eligible(spec, x, out, res):
            self.emit_convT_s2(x, spec, out, relu, tag)
            return
        if spec.kind == "convT" and 1 < len(spec.taps) <= 4:
            # the parity classes write disjoint output pixels: one grouped launch (no tail per class)
            probs = [dict(x=ptr(x.t), x_cs=x.cs, x_co=x.co, B=x.B, Hi=x.H, Wi=x.W, cin_p=spec.cin_p, Hg=x.H, Wg=x.W,
                          in_s=1, taps=taps, wt=ptr(spec.wt[cls]), N=np_, n_store=np_, scale=ptr(spec.scale),
                          bias=ptr(spec.bias), res=ptr(res.t) if res is not None else None,
                          res_cs=res.cs if res is not None else 0, res_co=res.co if res is not None else 0,
                          out=ptr(out.t), out_cs=out.cs, out_co=out.co, Ho=out.H, Wo=out.W, osy=2, osx=2, ooy=ooy,
                          oox=oox, relu=relu, cin=spec.cin, cout=spec.cout)
                     for cls, (taps, (ooy, oox)) in enumerate(zip(spec.taps, spec.cls_off))]
            q = CONVT_KCHUNK if CONVT_KCHUNK and spec.cin_p % CONVT_KCHUNK == 0 else 0
            wts = [ops.kchunk_weights(w, len(t), spec.cin_p, q) for w, t in zip(spec.wt, spec.taps)] if q else spec.wt
            for pr in probs:
                pr["k_chunk"] = q
            for pr, cls in zip(probs, range(len(probs))):
                w3 = ops.conv_weights_x3(wts[cls])
                self.specs.append(w3)
                pr["wt"] = ptr(w3)
            # split-bf16: the 128x128x16 tile (profiles/bench_conv_x3.py: transposed 4x4 272 -> 128 at
            # 30 px 501 us, 3x3 128 -> 128 at 60 px 665 us, against 742 / 854 for the f32 64x64x32)
            add_conv_group(self.plan, probs, tile=1, tag=tag + "_convT", x3=True)
            return
        for cls, (taps, (ooy, oox)) in enumerate(zip(spec.taps, spec.cls_off)):
            if spec.kind == "conv":
                Hg, Wg, in_s, osy, osx = out.H, out.W, spec.stride, 1, 1
            else:
                Hg, Wg, in_s, osy, osx = x.H, x.W, 1, 2, 2
            w3 = ops.conv_weights_x3(spec.wt[cls])  # split-bf16 operands (f32 accuracy)
            self.specs.append(w3)
            add_conv(self.plan, x=ptr(x.t), x_cs=x.cs, x_co=x.co, B=x.B, Hi=x.H, Wi=x.W, cin_p=spec.cin_p, Hg=Hg,
                     Wg=Wg, in_s=in_s, taps=taps, wt=ptr(spec.wt[cls]), N=np_, n_store=np_, scale=ptr(spec.scale),
                     bias=ptr(spec.bias), res=ptr(res.t) if res is not None else None,
                     res_cs=res.cs if res is not None else 0, res_co=res.co if res is not None else 0,
                     out=ptr(out.t), out_cs=out.cs, out_co=out.co, Ho=out.H, Wo=out.W, osy=osy, osx=osx, ooy=ooy,
                     oox=oox, relu=relu, cin=spec.cin, cout=spec.cout, tag=tag, wt3=ptr(w3))

    def resize(self, x: Act, out: Act, add: Optional[Act] = None, align: bool = False, relu: bool = False):
        assert x.cp == out.cp
        self.plan.add("krrn_resize_bilinear_f32", ptr(x.t), x.B, x.H, x.W, x.cs, x.co, x.cp, ptr(out.t), out.H,
                      out.W, out.cs, out.co, ptr(add.t if add is not None else None),
                      add.cs if add is not None else 0, add.co if add is not None else 0, int(align), int(relu))

    def add_relu(self, a: Act, b: Optional[Act], out: Act, relu: bool = True):
        self.plan.add("krrn_add_relu_f32", ptr(a.t), a.cs, a.co, ptr(b.t if b is not None else None),
                      b.cs if b is not None else 0, b.co if b is not None else 0, ptr(out.t), out.cs, out.co,
                      a.B * a.H * a.W, a.cp, int(relu))

    # -- blocks ------------------------------------------------------------------------
    def basic(self, x: Act, blk: BasicBlock, out: Optional[Act] = None) -> Act:
        h = self.conv(x, blk.conv1, blk.bn1, relu=True)
        res = x if blk.downsample is None else self.conv(x, blk.downsample[0], blk.downsample[1])
        return self.conv(h, blk.conv2, blk.bn2, out=out, res=res, relu=True)

    def bottleneck(self, x: Act, blk: Bottleneck) -> Act:
        h = self.conv(x, blk.conv1, blk.bn1, relu=True)
        h = self.conv(h, blk.conv2, blk.bn2, relu=True)
        res = x if blk.downsample is None else self.conv(x, blk.downsample[0], blk.downsample[1])
        return self.conv(h, blk.conv3, blk.bn3, res=res, relu=True)

    def hr_module(self, xs: List[Act], m: HighResolutionModule, outs: Optional[List[Optional[Act]]] = None,
                  fork_in: bool = True, join_out: bool = True) -> List[Act]:
        """myhrnet.py:226-250. Branch i (and later fuse output i) runs on plan stream i: the
        branches are independent until the fuse, and the fuse outputs are independent again.
        fork_in = False: xs[i] was produced on stream i (the previous module's fuse output i), so
        branch i needs no fork from stream 0; join_out = False: the outputs stay on their streams for
        the next module (the caller joins after the last one)."""
        plan = self.plan
        nb = m.num_branches
        side = list(range(1, nb))
        pre = {}
        ys = []
        if fork_in:
            plan.fork(side)
        for i, x in enumerate(xs):
            with plan.on_stream(i):
                y = x
                for blk in m.branches[i]:
                    y = self.basic(y, blk)
                if nb > 1 and FUSE_EARLY:
                    pre.update(self._fuse_terms_from(y, m, i))
            ys.append(y)
        if not FUSE_EDGES or nb == 1:
            plan.join(side)
        if nb == 1:
            return ys
        fused = []
        if FUSE_EDGES:
            # fuse output i (stream i) waits for exactly the branches it reads (all of them, each
            # with its early terms), not for a join of every branch into stream 0 and a fork back
            for i in range(nb):
                for j in range(nb):
                    if j != i:
                        plan.edge(j, i)
        else:
            plan.fork(side)
        for i in range(nb):
            with plan.on_stream(i):
                fused.append(self._fuse_output(ys, m, i, outs[i] if outs is not None else None, pre))
        if join_out:
            plan.join(side)
        return fused

    def _fuse_terms_from(self, y: Act, m: HighResolutionModule, j: int) -> dict:
        """The fuse-layer work that reads only branch j's output y (myhrnet.py:177-225), keyed by
        (output i, j): for i < j the 1x1 conv + BN at branch j's resolution (upsampled and added by
        _fuse_output), for i > j the stride-2 chain but its last conv (which adds into output i).
        Emitted on branch j's stream right after its blocks: the same launches as _fuse_output's own
        (bit-identical results), started before the other branches have finished."""
        terms = {}
        for i in range(m.num_branches):
            if i < j:
                seq = m.fuse_layers[i][j]
                terms[(i, j)] = self.conv(y, seq[0], seq[1])
            elif i > j:
                h = y
                for sub in m.fuse_layers[i][j][:-1]:
                    h = self.conv(h, sub[0], sub[1], relu=True)
                terms[(i, j)] = h
        return terms

    def _fuse_output(self, ys: List[Act], m: HighResolutionModule, i: int, out: Optional[Act],
                     pre: Optional[dict] = None) -> Act:
        """relu(sum_j fuse_layers[i][j](ys[j])) (myhrnet.py:232-248). With FUSE_ID_FIRST the identity
        term opens the sum (read in place) and every other term adds it in its producer's epilogue
        (conv residual / resize add), so no separate add launch exists; the f32 summation order then
        differs from the reference's j order (rounding-level)."""
        nb = m.num_branches
        out = out if out is not None else self.act(ys[i].H, ys[i].W, ys[i].c)
        acc: Optional[Act] = None  # running sum lives in `out` once written
        order = ([i] + [j for j in range(nb) if j != i]) if FUSE_ID_FIRST else list(range(nb))
        for pos, j in enumerate(order):
            last = pos == nb - 1
            if j == i:
                if acc is None:
                    acc = ys[i]  # identity term: read in place, no copy
                else:
                    self.add_relu(acc, ys[i], out, relu=last)
                    acc = out
            elif j > i:
                seq = m.fuse_layers[i][j]
                low = pre[(i, j)] if pre and (i, j) in pre else self.conv(ys[j], seq[0], seq[1])
                self.resize(low, out, add=acc, align=False, relu=last)
                acc = out
            else:
                chain = m.fuse_layers[i][j]
                h, first = (pre[(i, j)], len(chain) - 1) if pre and (i, j) in pre else (ys[j], 0)
                for k in range(first, len(chain)):
                    sub = chain[k]
                    if k == len(chain) - 1:
                        h = self.conv(h, sub[0], sub[1], out=out, res=acc, relu=last)
                    else:
                        h = self.conv(h, sub[0], sub[1], relu=True)
                acc = out
        return out


def build_hrnet_plan(net: HRNet, plan: Plan, x: Act, after_layer1=None) -> Tuple[Act, Act, list]:
    """Emit the HRNet forward (myhrnet.py:471-527) for input act `x`; returns (x_out @S/4, y_out @S/2).
    after_layer1(): called once the stem and layer1 are emitted (the caller forks side-stream work
    there, beside the latency-bound branch stages rather than the chip-filling stem)."""
    bld = _Builder(plan, x.B)
    h = bld.conv(x, net.conv1, net.bn1, relu=True)
    h = bld.conv(h, net.conv2, net.bn2, relu=True)
    for blk in net.layer1:
        h = bld.bottleneck(h, blk)
    if after_layer1 is not None:
        after_layer1()
    ylist = [h]
    nstages = len(net.spec.stages)
    on_streams = False  # ylist[k] lives on plan stream k (the previous stage was not joined)
    for si in range(nstages):
        trans = getattr(net, f"transition{si + 1}")
        stage = getattr(net, f"stage{si + 2}")
        nb = net.stage_branches[si]
        # per-stream stages: every module of the stage chains per stream (the grouped form runs on
        # stream 0, so not with it)
        cross = STAGE_STREAMS and MODULE_STREAMS and all(m.num_branches > 1 for m in stage)
        if on_streams and not cross:
            # the previous stage left branch k on stream k, but this stage runs its transitions on
            # stream 0 and forks from it: join first (not reached with W18 / W32 / W48, where every
            # stage after the first cross one is cross too; a custom spec with a 1-branch module is)
            plan.join(list(range(1, len(ylist))))
            on_streams = False
        xl = []
        for i in range(nb):
            t = trans[i]
            if t is None:
                if cross and not on_streams:
                    plan.sync(0, i)  # the previous stage was joined into stream 0
                xl.append(ylist[i])  # on stream i (on_streams) or joined into stream 0
            else:
                # myhrnet.py:482-507: transition1 reads the stem output; transition2 reads
                # y_list[-1] for every non-None entry; transition3 reads y_list[i] for
                # i < NUM_BRANCHES(stage3) and y_list[-1] otherwise.
                if si == 0:
                    k = 0
                elif si == 1:
                    k = len(ylist) - 1
                else:
                    k = i if i < len(ylist) else len(ylist) - 1
                src = ylist[k]
                chain = [t] if isinstance(t[0], nn.Conv2d) else list(t)
                sid = i if cross else 0
                if cross:
                    plan.sync(k if on_streams else 0, i)
                with plan.on_stream(sid):
                    for sub in chain:
                        src = bld.conv(src, sub[0], sub[1], relu=True)
                xl.append(src)
        last_stage = si == nstages - 1
        for mi, m in enumerate(stage):
            chain = MODULE_STREAMS and m.num_branches > 1
            fork_in = not chain or (mi == 0 and not cross)
            join_out = not chain or (mi == len(stage) - 1 and (last_stage or not cross))
            xl = bld.hr_module(xl, m, fork_in=fork_in, join_out=join_out)
        on_streams = cross and not last_stage
        ylist = xl
    # upsample + concat (myhrnet.py:511-516) straight into channel slices
    H0, W0 = ylist[0].H, ylist[0].W
    widths = [y.c for y in ylist]
    offs, o = [], 0
    for w in widths:
        offs.append(o)
        o += pad4(w)
    Lp = o
    L = sum(widths)
    # concat buffer: [cat(y0..y3) (Lp physical) | last_layer_1 out (L) | last_layer_2 out (C_b)]
    Cb = net.backbone_outc
    cat = bld.act(H0, W0, Lp, cs=Lp)
    for k, y in enumerate(ylist):
        dst = cat.slice(offs[k], y.c)
        if k == 0:
            bld.add_relu(y, None, dst, relu=False)
        else:
            bld.resize(y, dst, align=False)
    cat_map = []
    for k, w in enumerate(widths):
        cat_map += list(range(offs[k], offs[k] + w))
    # last_layer: conv3x3 'same' + bias + BN + ReLU (L -> L), then conv1x1 + bias (L -> C_b);
    # y = cat(x_list) = [last_layer_1 out, last_layer_2 out] (myhrnet.py:518-522)
    Lpp = pad4(L)
    ycat = bld.act(H0, W0, Lpp + pad4(Cb), cs=Lpp + pad4(Cb))
    x1 = ycat.slice(0, L)
    n0 = len(bld.specs)
    bld.conv(cat, net.last_layer[0][0], net.last_layer[0][1], out=x1, relu=True, cin_map=cat_map)
    x2 = ycat.slice(Lpp, Cb)
    bld.conv(x1, net.last_layer[1], None, out=x2, relu=False)
    if DECONV_FOLD and Lpp > L:
        # deconv(cat(x1, x2)) with x2 = W2 x1 + b2 (last_layer_2 is linear, myhrnet.py:339-345) ==
        # a transposed conv on [x1 | 1] alone: W_eff = W_a + W2^T W_b per tap, and the constant
        # channel carries W_b^T b2 (exact at the borders too: the ones channel is out of range
        # exactly where x2 would be). 272 instead of 400 input channels per tap (-32 % FLOPs).
        # The ones channel is x1's first pad channel, written by last_layer_1's epilogue with
        # scale 0 / bias 1 (its weight rows are zero) and read with zero weight by last_layer_2.
        bld.specs[n0].bias[L] = 1.0
        dc = net.deconv_layer[0][0]
        w = dc.weight.detach().double().cpu()  # [L + Cb, Cb_out, 4, 4]
        w2 = net.last_layer[1].weight.detach().double().cpu()[:, :, 0, 0]  # [Cb, L]
        b2 = net.last_layer[1].bias.detach().double().cpu()
        wa, wb = w[:L], w[L:L + Cb]
        w_eff = wa + torch.einsum("ci,cokl->iokl", w2, wb)
        w_one = torch.einsum("c,cokl->okl", b2, wb)[None]
        folded = nn.utils.skip_init(nn.ConvTranspose2d, L + 1, dc.out_channels, dc.kernel_size, dc.stride, dc.padding,
                                    bias=False)
        with torch.no_grad():
            folded.weight.copy_(torch.cat([w_eff, w_one]).float())
        x1o = Act(ycat.t, ycat.B, ycat.H, ycat.W, ycat.cs, 0, L + 1)
        d = bld.conv(x1o, folded, net.deconv_layer[0][1], relu=True)
    else:
        ycat_map = list(range(L)) + list(range(Lpp, Lpp + Cb))
        ycat_full = Act(ycat.t, ycat.B, ycat.H, ycat.W, ycat.cs, 0, Lpp + pad4(Cb))
        d = bld.conv(ycat_full, net.deconv_layer[0][0], net.deconv_layer[0][1], relu=True, cin_map=ycat_map)
    y = bld.basic(d, net.deconv_layer[1][0])
    return x2, y, bld.specs
