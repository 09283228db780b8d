"""Diagnostic for the intermittent graph-vs-serial mismatch of tests/test_gpu_pipeline.py::
test_pipelined_graph_benched_shape: the test's exact sequence (plain step + API forward, plain freed,
PipelinedPipeline eager half-step, capture, seed reset + stage-A reset + graph half-step), then slot 0's
stage B re-run serially from the same state; every slot-0 plan buffer that differs between the graph
half-step and the serial re-run is printed in allocation order with the first op touching it.

usage (GPU box): python3 profiles/race_bench_shape.py [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, get_pose, make_config  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.runtime import Op  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
if os.environ.get("HISTORY"):
    # the history under which the test fails: the other tests of tests/test_gpu_pipeline.py first
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    import test_gpu_pipeline as tgp  # noqa: E402
    for name, args in (("test_pipeline_matches_api_and_graph", (1,)), ("test_pipeline_matches_api_and_graph", (2,)),
                       ("test_pipelined_matches_plain", ("backbone",)), ("test_pipelined_matches_plain", ("heads",)),
                       ("test_pipelined_matches_plain", ("pose",)),
                       ("test_pipelined_matches_plain_after_history", ("heads",)),
                       ("test_pipelined_matches_plain_after_history", ("backbone",))):
        try:
            getattr(tgp, name)(dev, *args)
            print(f"{name}{args}: ok", flush=True)
        except AssertionError as e:
            print(f"{name}{args}: MISMATCH {str(e)[:120]}", flush=True)
    torch.cuda.synchronize()
B, S, N = 64, 120, 1000
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=1)
plain = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
plain.load(d)
plain.run()
torch.cuda.synchronize()
ref = {k: v.clone() for k, v in plain.results().items()}
pt = plain.parts[0]
perms = [pt.kp.perms[k].clone() for k, _, _ in pt.kp.perm_sizes]
out = m(d["img_croped"].to(dev), d["cloud"].to(dev), d["choose"].to(dev), d["cls_id"].to(dev), perms=perms)
R, t = get_pose(out, d, sel=pt.aux["sel"].clone(), subsets=pt.aux["subsets"].clone())
torch.cuda.synchronize()
del out, plain, pt
pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")
pp.load(d)
s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]
pp.run()
torch.cuda.synchronize()
pp.capture()

slot = pp.slots[0]
bufs, first = [], {}
for plan, _ in slot.plans():
    ts = [x for x in plan.buffers if isinstance(x, torch.Tensor)]
    for oi, op in enumerate(plan.ops):
        if not isinstance(op, Op):
            continue
        for a in op.args:
            v = getattr(a, "value", None)
            if v:
                for x in ts:
                    lo = x.data_ptr()
                    if lo <= v < lo + x.numel() * x.element_size() and lo not in first:
                        first[lo] = (oi, op.name, op.sid)
    bufs += ts

for rep in range(REPS):  # noqa: C901
    for sl, s in zip(pp.slots, s0):
        sl.parts[0].kp.seed.copy_(s)
    pp.reset()
    pp.step()
    torch.cuda.synchronize()
    got = {k: v.clone() for k, v in pp.results().items()}
    bad = [k for k in ref if not torch.equal(got[k], ref[k])]
    snap_g = [x.clone() for x in bufs]
    # slot 0's stage B again, serially, from the same state (stage A outputs are unchanged)
    slot.parts[0].kp.seed.copy_(s0[0])
    pp._run_b(0)
    torch.cuda.synchronize()
    snap_s = [x.clone() for x in bufs]
    diff = [i for i in range(len(bufs)) if not torch.equal(snap_g[i], snap_s[i])]
    print(f"rep {rep}: results differ from the plain step in {bad}; {len(diff)} slot-0 buffers differ "
          f"graph vs serial", flush=True)
    kp = slot.parts[0].kp
    named = dict(p9=kp.p9, xyz=kp.xyz, normal=kp.normal, **{k: v for k, v in kp.fusion_bufs.items()
                                                             if isinstance(v, torch.Tensor)})
    gsnap = {}
    for k, v in named.items():
        for i, x in enumerate(bufs):
            if x.data_ptr() == v.data_ptr():
                gsnap[k] = (snap_g[i], snap_s[i])
    for k, (gv, sv) in gsnap.items():
        if not torch.equal(gv, sv):
            dd = (gv != sv)
            if k == "F0":
                for sl3 in range(3):
                    part = dd[..., 128 * sl3:128 * (sl3 + 1)]
                    print(f"     F0 slice {sl3}: {int(part.sum())} entries differ, points "
                          f"{int(part.any(-1).sum())} of {part.shape[0] * part.shape[1]}", flush=True)
            print(f"     named {k}: {int(dd.sum())} entries differ of {dd.numel()}", flush=True)
    for i in diff[:12]:
        a, b = snap_s[i], snap_g[i]
        md = float((a.double() - b.double()).abs().max()) if a.is_floating_point() else int((a != b).sum())
        rows = ""
        if a.dim() >= 2:
            rb = (a != b).reshape(a.shape[0], -1).any(1).nonzero().flatten().tolist()
            rows = f" rows(dim0) {rb[:8]}"
        print(f"   buf {i} {tuple(a.shape)} {a.dtype} first op {first.get(bufs[i].data_ptr())} maxdiff {md:.3e}{rows}",
              flush=True)
