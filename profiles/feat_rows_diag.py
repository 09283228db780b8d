"""Which fusion feature rows miss FEAT_RTOL in test_forward_parity_configs[w32-1-1-320-4096-cat], and
why (diagnostic, not a test). Runs the HIP path and the oracle (conditioned on the HIP kNN picks over
predicted coordinates, as the test does) and prints, per failing row: the column block of its worst
error (fm5 0-511 level 2, feat1 512-895 level 0 v / x / n, feat2 896-1279 level 1), the error, and the
distance from the point's predicted xyz / normal to its nearest other point in that space (a level-0
surface conv normalises v_j - v_i: near-coincident predicted points amplify f32 noise).

usage (GPU box): python3 profiles/feat_rows_diag.py   (KRRN_CONVT_S2=0/1 to compare kernels)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.krrn_oracle import KRRNOracle  # noqa: E402
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.fusion import level_sizes  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

dev = torch.device("cuda", 0)
torch.set_num_threads(8)
B, S, N, C = 1, 320, 4096, 1
cfg = make_config(num_cls=C, backbone="w32")
m = KRRN(cfg=cfg)
sd = init_weights(m, 1)
m = m.to(dev).eval()
o = KRRNOracle(num_cls=C, backbone="w32")
o.load_state_dict(sd)
o.eval()
d = make_batch(B, S, N, seed=5)
d["cls_id"] = ((torch.arange(B) + 1) % C).view(B, 1)
g = torch.Generator().manual_seed(11)
N1, N2, _, _ = level_sizes(N, 10)
perms = [torch.randperm(N, generator=g)[:N1] for _ in range(4)] + [torch.randperm(N1, generator=g)[:N2]]
m.keep_fusion_feat = True
m.invalidate_plans()
out = m(d["img_croped"].to(dev), d["cloud"].to(dev), d["choose"].to(dev), d["cls_id"].to(dev),
        perms=[p.to(dev) for p in perms])
torch.cuda.synchronize()
plan = m.get_plan(B, S, N, True)
fb = plan.fusion_bufs
override = {br: fb[f"pool_{br}"].cpu() for br in ("v", "x", "n")}
override["idx2"] = fb["idx2"].cpu()
tr = {}
o(d["img_croped"], d["cloud"], d["choose"], d["cls_id"], perms=perms, trace=tr, pool_override=override)
fr = tr["feat"][..., :1280]
feat = plan.feat.cpu()
err = (feat - fr).abs() / fr.abs().max()
row = err.amax(-1)
bad = (row >= 1e-3).nonzero().tolist()
p9 = plan.p9.cpu()
print(f"lib convT_s2={os.environ.get('KRRN_CONVT_S2', '1')} rows {row.numel()} failing {len(bad)} max {float(row.max()):.2e}")
for b, p in bad:
    col = int(err[b, p].argmax())
    blk = "fm5" if col < 512 else ("feat1_" + "vxn"[(col - 512) // 128] if col < 896 else "feat2")
    dist = []
    for c0 in (3, 6):
        q = p9[b, :, c0:c0 + 3]
        dd = (q - q[p]).norm(dim=-1)
        dd[p] = float("inf")
        dist.append(float(dd.min() / q.norm(dim=-1).max()))
    print(f"  crop {b} point {p}: col {col} ({blk}) err {float(row[b, p]):.2e} "
          f"nearest other point / scale: xyz {dist[0]:.1e} normal {dist[1]:.1e}")
