"""ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product package (pose_estimation_amd/) never does.

A PyTorch-CPU (f32, eval) restatement of the KRRN inference path of yaomy533/pose_estimation,
written from the reference's behaviour, op for op:
  HRNet            lib/network/hrnet/myhrnet.py:34-527 (+ configs/hrnet_*.yaml)
  KRRN heads       lib/network/krrn.py:46-165
  FusionNetLite    lib/network/point/fusion.py:137-240, gcn3d.py:15-242
  TBase            lib/network/pose/posenet.py:51-96
  get_pose         tools/trainer.py:383-438 (PnP through oracle/pnp_ref.c)
Module attribute names are the reference's so that one state dict loads into this oracle,
into the product model and into a reference checkpoint alike.

Pinning (DESIGN.md "Parity"): importing/running the reference in this container was refused
 and the reference ships no tests, golden vectors or checkpoints, so this
restatement is PARITY UNPINNED against reference outputs. It is pinned where it can be:
kNN by hand-checkable known answers, PnP by exact-recovery known answers, bilinear/conv/BN by
torch's own operators (the reference's building blocks), and the whole forward by the
committed golden fixtures tests/golden/*.npz generated from it (tests/golden/make_golden.py).

Two places fix what the reference leaves implementation-defined, identically in the HIP path:
  * kNN distance expression order: inner products and squared norms are summed
    sequentially over the coordinate axis with every op rounded to f32 (the reference uses
    torch.bmm + sum, whose accumulation order is a BLAS detail), and
  * topk ties: the lower index wins (torch.topk leaves tie order unspecified).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))
_CFG_DIR = os.path.join(os.path.dirname(_HERE), "pose_estimation_amd", "configs")


# ----------------------------------------------------------------------------------------
# HRNet (myhrnet.py)
# ----------------------------------------------------------------------------------------

class BasicBlock(nn.Module):
    def __init__(self, cin, c, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(c, momentum=0.1)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(c, c, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(c, momentum=0.1)
        self.downsample = downsample

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        res = x if self.downsample is None else self.downsample(x)
        return self.relu(out + res)


class Bottleneck(nn.Module):
    def __init__(self, cin, c, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(c, momentum=0.1)
        self.conv2 = nn.Conv2d(c, c, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(c, momentum=0.1)
        self.conv3 = nn.Conv2d(c, 4 * c, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(4 * c, momentum=0.1)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        res = x if self.downsample is None else self.downsample(x)
        return self.relu(out + res)


class HRModule(nn.Module):
    def __init__(self, nb, blocks, inch, widths):
        super().__init__()
        self.nb = nb
        inch = list(inch)
        br = []
        for i in range(nb):
            ds = None
            if inch[i] != widths[i]:
                ds = nn.Sequential(nn.Conv2d(inch[i], widths[i], 1, 1, bias=False), nn.BatchNorm2d(widths[i]))
            layers = [BasicBlock(inch[i], widths[i], 1, ds)]
            inch[i] = widths[i]
            layers += [BasicBlock(inch[i], widths[i]) for _ in range(1, blocks[i])]
            br.append(nn.Sequential(*layers))
        self.branches = nn.ModuleList(br)
        self.out_ch = inch
        if nb > 1:
            rows = []
            for i in range(nb):
                row = []
                for j in range(nb):
                    if j > i:
                        row.append(nn.Sequential(nn.Conv2d(inch[j], inch[i], 1, 1, 0, bias=False), nn.BatchNorm2d(inch[i])))
                    elif j == i:
                        row.append(None)
                    else:
                        chain = []
                        for k in range(i - j):
                            if k == i - j - 1:
                                chain.append(nn.Sequential(nn.Conv2d(inch[j], inch[i], 3, 2, 1, bias=False),
                                                           nn.BatchNorm2d(inch[i])))
                            else:
                                chain.append(nn.Sequential(nn.Conv2d(inch[j], inch[j], 3, 2, 1, bias=False),
                                                           nn.BatchNorm2d(inch[j]), nn.ReLU(True)))
                        row.append(nn.Sequential(*chain))
                rows.append(nn.ModuleList(row))
            self.fuse_layers = nn.ModuleList(rows)
        else:
            self.fuse_layers = None
        self.relu = nn.ReLU(True)

    def forward(self, x: List[torch.Tensor]):
        if self.nb == 1:
            return [self.branches[0](x[0])]
        x = [self.branches[i](x[i]) for i in range(self.nb)]
        out = []
        for i in range(self.nb):
            y = x[0] if i == 0 else self.fuse_layers[i][0](x[0])
            for j in range(1, self.nb):
                if i == j:
                    y = y + x[j]
                elif j > i:
                    y = y + F.interpolate(self.fuse_layers[i][j](x[j]), size=[x[i].shape[-2], x[i].shape[-1]],
                                          mode="bilinear", align_corners=False)
                else:
                    y = y + self.fuse_layers[i][j](x[j])
            out.append(self.relu(y))
        return out


class HRNet(nn.Module):
    def __init__(self, spec, outc):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 3, 2, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.conv2 = nn.Conv2d(64, 64, 3, 2, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(True)
        ds = nn.Sequential(nn.Conv2d(64, 256, 1, 1, bias=False), nn.BatchNorm2d(256))
        self.layer1 = nn.Sequential(Bottleneck(64, 64, 1, ds), Bottleneck(256, 64), Bottleneck(256, 64),
                                    Bottleneck(256, 64))
        pre = [256]
        self.nbr = []
        for si, st in enumerate(spec["stages"]):
            w = list(st["widths"])
            trans = []
            for i in range(len(w)):
                if i < len(pre):
                    trans.append(None if w[i] == pre[i] else nn.Sequential(
                        nn.Conv2d(pre[i], w[i], 3, 1, 1, bias=False), nn.BatchNorm2d(w[i]), nn.ReLU(True)))
                else:
                    chain = []
                    for j in range(i + 1 - len(pre)):
                        cout = w[i] if j == i - len(pre) else pre[-1]
                        chain.append(nn.Sequential(nn.Conv2d(pre[-1], cout, 3, 2, 1, bias=False), nn.BatchNorm2d(cout),
                                                   nn.ReLU(True)))
                    trans.append(nn.Sequential(*chain))
            setattr(self, f"transition{si + 1}", nn.ModuleList(trans))
            mods, inch = [], list(w)
            for _ in range(st["modules"]):
                m = HRModule(len(w), st["blocks"], inch, w)
                mods.append(m)
                inch = m.out_ch
            setattr(self, f"stage{si + 2}", nn.Sequential(*mods))
            pre = inch
            self.nbr.append(len(w))
        L = sum(pre)
        self.last_layer = nn.ModuleList([
            nn.Sequential(nn.Conv2d(L, L, 3, 1, padding="same"), nn.BatchNorm2d(L), nn.ReLU(True)),
            nn.Conv2d(L, outc, 1, 1, 0)])
        self.deconv_layer = nn.ModuleList([
            nn.Sequential(nn.ConvTranspose2d(L + outc, outc, 4, 2, 1, bias=False), nn.BatchNorm2d(outc), nn.ReLU(True)),
            nn.Sequential(BasicBlock(outc, outc))])

    def forward(self, x):
        x = self.relu(self.bn1(self.conv1(x)))
        x = self.relu(self.bn2(self.conv2(x)))
        x = self.layer1(x)
        y = [x]
        for si, nb in enumerate(self.nbr):
            trans = getattr(self, f"transition{si + 1}")
            xl = []
            for i in range(nb):
                if trans[i] is None:
                    xl.append(y[i])
                elif si == 0:
                    xl.append(trans[i](y[0]))
                elif si == 1:
                    xl.append(trans[i](y[-1]))
                else:
                    xl.append(trans[i](y[i] if i < len(y) else y[-1]))
            y = getattr(self, f"stage{si + 2}")(xl)
        h, w = y[0].shape[2], y[0].shape[3]
        ups = [y[0]] + [F.interpolate(t, size=(h, w), mode="bilinear", align_corners=False) for t in y[1:]]
        x = torch.cat(ups, 1)
        outs = []
        for layer in self.last_layer:
            x = layer(x)
            outs.append(x)
        z = torch.cat(outs, 1)
        for layer in self.deconv_layer:
            z = layer(z)
        return x, z


# ----------------------------------------------------------------------------------------
# 3D-GCN (gcn3d.py) with the fixed expression order / tie rule
# ----------------------------------------------------------------------------------------

def _seq_sum(p: torch.Tensor) -> torch.Tensor:
    s = p[..., 0]
    for i in range(1, p.shape[-1]):
        s = s + p[..., i]
    return s


def _stable_topk_small(dist: torch.Tensor, k: int) -> torch.Tensor:
    return torch.sort(dist, dim=-1, stable=True)[1][..., :k]


def neighbor_dist(v: torch.Tensor) -> torch.Tensor:
    """gcn3d.py:21-23: -2 <vi, vj> + |vj|^2 + |vi|^2 (rows i = queries)."""
    inner = _seq_sum(v[:, :, None, :] * v[:, None, :, :])
    q = _seq_sum(v * v)
    return (inner * -2.0 + q[:, None, :]) + q[:, :, None]


def get_neighbor_index(v: torch.Tensor, k: int, rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """gcn3d.py:15-26 (rows: evaluate only these query rows; identical per-row result)."""
    d = neighbor_dist(v)
    if rows is not None:
        d = d[:, rows]
    return _stable_topk_small(d, k + 1)[..., 1:]


def get_nearest_index(target: torch.Tensor, source: torch.Tensor) -> torch.Tensor:
    """gcn3d.py:29-38: |s_j|^2 + |t_i|^2 - 2 <t_i, s_j>, k = 1."""
    inner = _seq_sum(target[:, :, None, :] * source[:, None, :, :])
    s2 = _seq_sum(source * source)
    t2 = _seq_sum(target * target)
    d = (s2[:, None, :] + t2[:, :, None]) - 2.0 * inner
    return _stable_topk_small(d, 1)


def indexing_neighbor(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    b = torch.arange(t.shape[0]).view(-1, 1, 1)
    return t[b, idx]


def direction_norm(v, idx):
    return F.normalize(indexing_neighbor(v, idx) - v.unsqueeze(2), dim=-1)


class Conv_surface(nn.Module):  # noqa: N801
    def __init__(self, kernel_num, support_num):
        super().__init__()
        self.kernel_num, self.support_num = kernel_num, support_num
        self.relu = nn.ReLU(True)
        self.directions = nn.Parameter(torch.empty(3, support_num * kernel_num))
        s = 1.0 / math.sqrt(support_num * kernel_num)
        nn.init.uniform_(self.directions, -s, s)

    def forward(self, idx, v):
        bs, n, k = idx.shape
        th = self.relu(direction_norm(v, idx) @ F.normalize(self.directions, dim=0))
        th = th.view(bs, n, k, self.support_num, self.kernel_num)
        return torch.max(th, dim=2)[0].sum(dim=2)


class Conv_layer(nn.Module):  # noqa: N801
    dim = 3

    def __init__(self, cin, cout, support_num):
        super().__init__()
        self.in_channel, self.out_channel, self.support_num = cin, cout, support_num
        self.relu = nn.ReLU(True)
        self.weights = nn.Parameter(torch.empty(cin, (support_num + 1) * cout))
        self.bias = nn.Parameter(torch.empty((support_num + 1) * cout))
        self.directions = nn.Parameter(torch.empty(self.dim, support_num * cout))
        s = 1.0 / math.sqrt(cout * (support_num + 1))
        for p in (self.weights, self.bias, self.directions):
            nn.init.uniform_(p, -s, s)

    def forward(self, idx, v, fm):
        bs, n, k = idx.shape
        th = self.relu(direction_norm(v, idx) @ F.normalize(self.directions, dim=0))
        out = fm @ self.weights + self.bias
        c = self.out_channel
        center, support = out[:, :, :c], out[:, :, c:]
        act = th * indexing_neighbor(support, idx)
        act = act.view(bs, n, k, self.support_num, c)
        return center + torch.max(act, dim=2)[0].sum(dim=2)


class Conv_fuse_layer(Conv_layer):  # noqa: N801
    dim = 9


class Pool_layer(nn.Module):  # noqa: N801
    def __init__(self, pooling_rate=4, neighbor_num=4):
        super().__init__()
        self.pooling_rate, self.neighbor_num = pooling_rate, neighbor_num

    def forward(self, v, fm, perm=None, idx_override=None):
        """idx_override (test conditioning): use these neighbour indices for the max instead of
        the kNN result (which is still computed and kept in `last_idx`)."""
        n = v.shape[1]
        pool_num = int(n / self.pooling_rate)
        sample = torch.randperm(n)[:pool_num] if perm is None else perm[:pool_num].long()
        idx = get_neighbor_index(v[..., :3], self.neighbor_num, rows=sample)
        self.last_idx = idx
        if idx_override is not None:
            idx = idx_override.long()
        pooled = torch.max(indexing_neighbor(fm, idx), dim=2)[0]
        return v[:, sample, :], pooled, sample


class FusionNetLite(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.neighbor_num = cfg["GCN_N_NUM"]
        self.support_num = S = cfg["GCN_SUP_NUM"]
        for br in ("v", "x", "n"):
            setattr(self, f"conv_0_{br}", Conv_surface(128, S))
            setattr(self, f"conv_1_{br}", Conv_layer(128, 128, S))
            setattr(self, f"pool_1_{br}", Pool_layer())
            setattr(self, f"conv_2_{br}", Conv_layer(128, 128, S))
            setattr(self, f"bn1_{br}", nn.BatchNorm1d(128))
            setattr(self, f"bn2_{br}", nn.BatchNorm1d(128))
        self.pool_1 = Pool_layer()
        self.pool_2 = Pool_layer()
        self.conv_4 = Conv_fuse_layer(384, 512, S)
        self.conv_5 = Conv_fuse_layer(512, 512, S)

    @staticmethod
    def _bnr(bn, x):
        return F.relu(bn(x.transpose(1, 2)).transpose(1, 2))

    def forward(self, vertices, xyz, normal, perms: Optional[Sequence[torch.Tensor]] = None, trace=None,
                pool_override=None):
        perms = list(perms) if perms is not None else [None] * 5
        k0 = self.neighbor_num
        idx0 = get_neighbor_index(vertices, k0)
        pts = {"v": vertices, "x": xyz, "n": normal}
        fm1 = {}
        for br in ("v", "x", "n"):
            f0 = F.relu(getattr(self, f"conv_0_{br}")(idx0, pts[br]))
            fm1[br] = self._bnr(getattr(self, f"bn1_{br}"), getattr(self, f"conv_1_{br}")(idx0, pts[br], f0))
        feat_1 = torch.cat([fm1["v"], fm1["x"], fm1["n"]], 2)
        feat_feature = torch.cat([vertices, xyz, normal], 2)
        vp, fp, used = {}, {}, []
        for i, br in enumerate(("v", "x", "n")):
            ov = pool_override.get(br) if pool_override else None
            vp[br], fp[br], s = getattr(self, f"pool_1_{br}")(pts[br], fm1[br], perms[i], idx_override=ov)
            used.append(s)
        pool_1, _, s = self.pool_1(feat_feature, feat_1, perms[3])
        used.append(s)
        k1 = min(k0, vp["v"].shape[1] // 8)
        idx1 = get_neighbor_index(vp["v"], k1)
        fm2 = [self._bnr(getattr(self, f"bn2_{br}"), getattr(self, f"conv_2_{br}")(idx1, vp[br], fp[br]))
               for br in ("v", "x", "n")]
        feat_2 = torch.cat(fm2, 2)
        pool_2, fm_pool_2, s = self.pool_2(pool_1, feat_2, perms[4])
        used.append(s)
        k2 = min(k0, pool_2.shape[1] // 8)
        idx2 = get_neighbor_index(pool_2, k2)
        idx2_used = pool_override["idx2"].long() if pool_override and "idx2" in pool_override else idx2
        fm_4 = self.conv_4(idx2_used, pool_2, fm_pool_2)
        fm_5 = self.conv_5(idx2_used, pool_2, fm_4)
        nn1 = get_nearest_index(vertices, pool_1[..., :3])
        nn2 = get_nearest_index(vertices, pool_2[..., :3])
        feat = torch.cat([indexing_neighbor(fm_5, nn2).squeeze(2), indexing_neighbor(feat_1, nn1).squeeze(2),
                          indexing_neighbor(feat_2, nn1).squeeze(2)], 2)
        if trace is not None:
            trace.update(idx0=idx0, idx1=idx1, idx2=idx2, nn1=nn1[..., 0], nn2=nn2[..., 0], feat1=feat_1, p9=feat_feature,
                         feat2=feat_2, fm5=fm_5, pool_1=pool_1, pool_2=pool_2, perms=used,
                         pool_v=self.pool_1_v.last_idx, pool_x=self.pool_1_x.last_idx,
                         pool_n=self.pool_1_n.last_idx, pool2=self.pool_2.last_idx)
        return feat


class TBase(nn.Module):
    def __init__(self, f, k=3):
        super().__init__()
        self.conv1 = nn.Conv1d(f, 1024, 1)
        self.conv2 = nn.Conv1d(1024, 256, 1)
        self.conv3 = nn.Conv1d(256, 256, 1)
        self.conv4 = nn.Conv1d(256, k, 1)
        self.drop1 = nn.Dropout(0.2)
        self.bn1 = nn.BatchNorm1d(1024)
        self.bn2 = nn.BatchNorm1d(256)
        self.bn3 = nn.BatchNorm1d(256)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.relu(self.bn2(self.conv2(x)))
        x = F.relu(self.bn3(self.conv3(x)))
        x = self.conv4(self.drop1(x))
        return x[:, 0:3]


class PoseNet(nn.Module):
    def __init__(self, f, k=3):
        super().__init__()
        self.t_net = TBase(f, k)


class KRRNOracle(nn.Module):
    """lib/network/krrn.py:27-165 on the CPU, f32."""

    def __init__(self, num_cls=1, backbone="w18", backbone_outc=128, head_fs=128, region_out=65, gcn_k=10, gcn_s=7,
                 inc_r=1280, out_t=3):
        super().__init__()
        with open(os.path.join(_CFG_DIR, f"hrnet_{backbone}.yaml")) as f:
            spec = yaml.safe_load(f)
        self.num_cls = C = num_cls
        self.backbone = HRNet(spec, backbone_outc)
        self.mask_outc = C + 1
        self.region_outc = self.mask_outc + region_out
        self.xyz_outc = self.region_outc + 3 * C
        F_ = head_fs

        def cbr(cin, cout):
            return [nn.Conv2d(cin, cout, 3, 1, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(True)]
        self.XYZNet = nn.Sequential(nn.ConvTranspose2d(backbone_outc, F_, 3, 2, 1, output_padding=1, bias=False),
                                    nn.BatchNorm2d(F_), nn.ReLU(True), *cbr(F_, F_),
                                    nn.UpsamplingBilinear2d(scale_factor=2.0), *cbr(F_, F_), *cbr(F_, F_))
        self.xyz_final = nn.Conv2d(F_, self.xyz_outc, 1)
        self.NMLNet = nn.Sequential(*cbr(backbone_outc, F_), *cbr(F_, F_), nn.UpsamplingBilinear2d(scale_factor=2.0),
                                    *cbr(F_, F_))
        self.nml_final = nn.Conv2d(F_, 3 * C, 1)
        self.fusion = FusionNetLite({"GCN_N_NUM": gcn_k, "GCN_SUP_NUM": gcn_s})
        self.pose = PoseNet(inc_r + C, out_t)

    @torch.no_grad()
    def forward(self, x, p_emb, choose, cls, region_point=None, opt_pose=True, perms=None, trace=None,
                pool_override=None):
        bs = x.size(0)
        xm, nm = self.backbone(x)
        xm = self.xyz_final(self.XYZNet(xm))
        nm = self.nml_final(self.NMLNet(nm))
        h, w = xm.shape[2], xm.shape[3]
        mask = xm[:, :self.mask_outc]
        region = xm[:, self.mask_outc:self.region_outc]
        xyz = xm[:, self.region_outc:self.xyz_outc]
        C = self.num_cls
        xyz = torch.gather(xyz.reshape(bs, C, 3, h, w), 1, cls.view(bs, 1, 1, 1, 1).repeat(1, 1, 3, h, w)).squeeze(1)
        nml = torch.gather(nm.reshape(bs, C, 3, h, w), 1, cls.view(bs, 1, 1, 1, 1).repeat(1, 1, 3, h, w)).squeeze(1)
        nml = F.normalize(nml, p=2, dim=1)
        out = {"xyz": xyz, "region": region, "mask": mask, "normal": nml, "pred_r": None, "pred_t": None}
        if not opt_pose:
            return out
        xe = torch.gather(xyz.reshape(bs, 3, -1), -1, choose.repeat(1, 3, 1)).permute(0, 2, 1)
        ne = torch.gather(nml.reshape(bs, 3, -1), -1, choose.repeat(1, 3, 1)).permute(0, 2, 1)
        feat = self.fusion(p_emb, xe, ne, perms=perms, trace=trace, pool_override=pool_override)
        n = p_emb.size(1)
        one_hot = torch.zeros(bs, C).scatter_(1, cls.view(-1, 1).long(), 1)
        feat = torch.cat([feat, one_hot.unsqueeze(1).repeat(1, n, 1)], 2)
        t_res = self.pose.t_net(feat.permute(0, 2, 1))
        out["pred_t"] = (p_emb + t_res.permute(0, 2, 1)).mean(dim=1)
        if trace is not None:
            trace.update(feat=feat, t_res=t_res)
        return out


def get_pose(pred, data, sel, subsets, thr=1.0):
    """tools/trainer.py:383-438 for every crop of the batch with explicit randomness.

    sel: [B, P] choose-subset indices (randperm(N)[:256] per crop); subsets: [B, H, 5].
    Returns (R [B,3,3] f32, t [B,3] f32, inlier counts [B])."""
    from . import pnp
    xyz = pred["xyz"].detach().cpu().double()
    B = xyz.shape[0]
    ext = data["extent"].double()
    lfb = data["lfborder"].double()
    choose = data["choose"].reshape(B, -1)
    Rs, ts, cnts = [], [], []
    for b in range(B):
        s = sel[b].long()
        pix = choose[b, s]
        coord = xyz[b].reshape(3, -1)[:, pix].t() * ext[b] + lfb[b]
        obj = coord.float().numpy()
        img = torch.stack([data["x_map_choosed"][b].reshape(-1)[s], data["y_map_choosed"][b].reshape(-1)[s]], 1)
        R, t, cnt, _, _ = pnp.pnp_ransac(obj, img.float().numpy(), data["intrinsic"][b].numpy(),
                                         subsets[b].numpy(), thr)
        Rs.append(torch.from_numpy(R))
        ts.append(torch.from_numpy(t))
        cnts.append(cnt)
    return torch.stack(Rs), torch.stack(ts), torch.tensor(cnts)
