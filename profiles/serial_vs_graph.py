"""Diagnostic: one KRRN forward plan run serially (every launch on the caller's stream) vs the same
plan captured with its side streams into a hipGraph and replayed, vs eager multi-stream. Prints
every plan buffer that differs, in allocation order, with the op that first writes it.

usage (GPU box): python3 profiles/serial_vs_graph.py [B S N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.runtime import Op, Sync  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

B, S, N = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (4, 120, 1000)
dev = torch.device("cuda", 0)
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=9)
g = torch.Generator().manual_seed(2)
N1 = N // 4
perms = [torch.randperm(N, generator=g)[:N1] for _ in range(4)] + [torch.randperm(N1, generator=g)[:N1 // 4]]
m(d["img_croped"].to(dev), d["cloud"].to(dev), d["choose"].to(dev), d["cls_id"].to(dev), perms=[p.to(dev) for p in perms])
torch.cuda.synchronize()
kp = m.get_plan(B, S, N, True)
plan = kp.plan
bufs = [t for t in plan.buffers if isinstance(t, torch.Tensor)]
# the first op (index, name, stream) whose argument lies inside each buffer
first = {}
for oi, op in enumerate(plan.ops):
    if not isinstance(op, Op):
        continue
    for a in op.args:
        v = getattr(a, "value", None)
        if not v:
            continue
        for bi, t in enumerate(bufs):
            lo = t.data_ptr()
            if lo <= v < lo + t.numel() * t.element_size() and bi not in first:
                first[bi] = (oi, op.name, op.sid)


def snap():
    return [t.clone() for t in bufs]


plan.run(kp.env)
torch.cuda.synchronize()
ser = snap()
plan.run(kp.env)
torch.cuda.synchronize()
ser2 = snap()
plan.run(kp.env, serial=False)
torch.cuda.synchronize()
eag = snap()
gr = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(gr, stream=s):
        plan.run(kp.env, serial=False)
torch.cuda.current_stream().wait_stream(s)
reps = int(os.environ.get("REPS", "1"))
gra = None
for r in range(reps):  # intermittent orderings: every replay must equal the serial run
    gr.replay()
    torch.cuda.synchronize()
    cur = snap()
    nbad = sum(not torch.equal(a, b) for a, b in zip(ser, cur))
    if reps > 1:
        print(f"replay {r}: {nbad} buffers differ", flush=True)
    if gra is None or nbad:
        gra = cur
print(f"plan: {len(plan.ops)} ops, {len(bufs)} buffers, streams {plan.nstreams}", flush=True)
for name, other in (("serial-again", ser2), ("eager-multistream", eag), ("graph", gra)):
    bad = [bi for bi in range(len(bufs)) if not torch.equal(ser[bi], other[bi])]
    print(f"{name}: {len(bad)} buffers differ from the serial run", flush=True)
    for bi in bad[:12]:
        a, b = ser[bi], other[bi]
        diff = float((a.double() - b.double()).abs().max()) if a.is_floating_point() else int((a != b).sum())
        print(f"   buf {bi} {tuple(a.shape)} {a.dtype} first op {first.get(bi)} maxdiff {diff:.3e}", flush=True)
