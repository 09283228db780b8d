"""Per-op serial device time of one bench step (HIP events around every plan op, eager, one
stream), grouped by kernel; fusion ops (G1-G9) listed one by one.

usage (GPU box): python3 profiles/op_table.py [out.json]   (env B, S, N, BB; KRRN_HIP_LIB to
time a kernel-variant build of the library)
"""
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd.config import make_config  # noqa: E402
from pose_estimation_amd.krrn import KRRN  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

B, S, N = int(os.environ.get("B", 64)), int(os.environ.get("S", 120)), int(os.environ.get("N", 1000))
dev = torch.device("cuda", 0)
m = KRRN(cfg=make_config(num_cls=1, backbone=os.environ.get("BB", "w18")))
init_weights(m, 0)
m = m.to(dev).eval()
m.perm_mode = "device"
st = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
st.load(make_batch(B, S, N, seed=1))
st.run()
torch.cuda.synchronize()
st.profile()
prof = st.profile()
fids = set().union(*(getattr(pt.kp, "fusion_op_ids", set()) for pt in st.parts))
rows, agg = [], defaultdict(lambda: [0.0, 0])
for op, ms in prof:
    tag = op.meta.get("tag", "")
    rows.append(dict(name=op.name, tag=tag, gf=op.meta.get("flops", 0) / 1e9, ms=ms, sid=op.sid,
                     fusion=id(op) in fids))
    a = agg[op.name + (f"[{tag}]" if tag else "")]
    a[0] += ms
    a[1] += 1
if len(sys.argv) > 1:
    json.dump(rows, open(sys.argv[1], "w"), indent=0)
print(f"lib={os.environ.get('KRRN_HIP_LIB', 'in-tree')} B={B} S={S} N={N} total {sum(r['ms'] for r in rows):.3f} ms")
for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"  {k:40s} {ms:8.3f} ms  x{n}")
fu = [r for r in rows if r["fusion"]]
print(f"fusion {sum(r['ms'] for r in fu):.3f} ms over {len(fu)} ops")
for r in fu:
    print(f"    {r['name']:26s} {r['tag']:10s} {r['ms'] * 1e3:8.1f} us sid={r['sid']}")
