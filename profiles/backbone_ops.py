"""Per-op serial device time of the HRNet backbone part of one plan (ops[:split]), with shapes,
grouped by (kernel, tag, M, N, K); and the same for the heads (ops[split:heads_end]) and the
tail (fusion + TBase, ops[heads_end:]; the PnP pose plan is separate).
usage (GPU box): python3 profiles/backbone_ops.py [B]"""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd.config import make_config  # noqa: E402
from pose_estimation_amd.krrn import KRRN  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, _sub_plan  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S, N = 120, 1000
dev = torch.device("cuda", 0)
m = KRRN(cfg=make_config(num_cls=1, backbone=os.environ.get("BB", "w18")))
init_weights(m, 0)
m = m.to(dev).eval()
m.perm_mode = "device"
st = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
st.load(make_batch(B, S, N, seed=1))
st.run()
torch.cuda.synchronize()
kp = st.parts[0].kp
for name, lo, hi in (("backbone", 0, kp.split), ("heads", kp.split, kp.heads_end),
                     ("tail", kp.heads_end, len(kp.plan.ops))):
    sub = _sub_plan(kp.plan, lo, hi)
    sub.run_timed(dict(kp.env))
    prof = sub.run_timed(dict(kp.env))
    tot = sum(t for _, t in prof)
    groups = defaultdict(lambda: [0.0, 0, 0.0])
    for op, t in prof:
        mt = op.meta
        key = (op.name, mt.get("kernel", ""), mt.get("tag", ""), mt.get("M"), mt.get("N"), mt.get("K"), mt.get("splits"))
        g = groups[key]
        g[0] += t
        g[1] += 1
        g[2] += mt.get("flops", 0.0)
    print(f"== {name}: {tot:.3f} ms serial over {len(prof)} launches")
    for key, (t, n, fl) in sorted(groups.items(), key=lambda kv: -kv[1][0])[:40]:
        tf = fl / (t * 1e-3) / 1e12 if fl else 0
        print(f"  {t:7.3f} ms x{n:3d} {t / n * 1e3:7.1f} us/launch {tf:6.1f} TF  {key}")
