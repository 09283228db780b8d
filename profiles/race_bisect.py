"""Diagnostic for the PipelinedPipeline(split='heads') vs plain mismatch.

Runs the given pytest files in-process first (the allocator history under which the mismatch was
seen), then compares slot 0 of one PipelinedPipeline half-step against the plain BatchPipeline
step of the same seed under several execution modes:

  concurrent   stage A(1) on the side stream beside stage B(0) (the bench's schedule)
  sequential   A(1) only after B(0) has finished
  b_serial     B(0) with every plan stream folded onto one stream, A(1) concurrent
  a_serial     A(1) folded onto one stream, B(0) concurrent with its own side streams
  no_a         B(0) alone

usage: python3 profiles/race_bisect.py REPS [pytest files ...]"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
if len(sys.argv) > 2:
    pytest.main(["-q", "-p", "no:cacheprovider", "-x"] + sys.argv[2:])
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

dev = torch.device("cuda", 0)
B, S, N = 4, 64, 256
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=22)


def bufs(kp):
    out = {"xyz": kp.xyz, "normal": kp.normal, "p9": kp.p9, "pred_t": kp.pred_t}
    out.update({f"perm_{k}": v for k, v in kp.perms.items()})
    for k, v in kp.fusion_bufs.items():
        for i, t in enumerate(v if isinstance(v, list) else [v]):
            if isinstance(t, torch.Tensor):
                out[f"fus_{k}" + (f"[{i}]" if isinstance(v, list) else "")] = t
    out.update({f"tb_{k}": v for k, v in kp.tbase_bufs.items() if isinstance(v, torch.Tensor)})
    return {k: v.clone() for k, v in out.items()}


plain = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
plain.load(d)
plain.run()
torch.cuda.synchronize()
ref = bufs(plain.parts[0].kp)
ref_res = {k: v.clone() for k, v in plain.results().items()}

pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")
pp.load(d)
s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]


def run_stage(stage, serial):
    for p, env in stage:
        p.run(dict(env), serial=serial)


def trial(mode):
    for sl, s in zip(pp.slots, s0):
        sl.parts[0].kp.seed.copy_(s)
    pp.reset()
    torch.cuda.synchronize()
    main = torch.cuda.current_stream(dev)
    side = pp.side
    a_stage, b_stage = pp.stage_a[1], pp.stage_b[0]
    if mode == "sequential":
        run_stage(b_stage, False)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            run_stage(a_stage, False)
        main.wait_stream(side)
    elif mode == "no_a":
        run_stage(b_stage, False)
    else:
        side.wait_stream(main)
        with torch.cuda.stream(side):
            run_stage(a_stage, mode == "a_serial")
        run_stage(b_stage, mode == "b_serial")
        main.wait_stream(side)
    torch.cuda.synchronize()
    got = bufs(pp.slots[0].parts[0].kp)
    diffs = [k for k in ref if not torch.equal(ref[k], got[k])]
    res = pp.slots[0].results()
    rdiff = [k for k in ref_res if not torch.equal(ref_res[k], res[k])]
    detail = ""
    if "fus_feat2" in diffs:
        a, b = ref["fus_feat2"], got["fus_feat2"]
        for bi in range(3):
            dd = (a[..., 128 * bi:128 * bi + 128] - b[..., 128 * bi:128 * bi + 128]).abs().amax(-1)
            if (dd > 0).any():
                rows = torch.nonzero(dd > 0).tolist()
                detail += f" feat2[{bi}] rows {rows[:6]} max {float(dd.max()):.2e};"
    return diffs, rdiff, detail


MODES = os.environ.get("MODES", "concurrent,sequential,b_serial,a_serial,no_a,graph").split(",")


def trial_graph():
    """The bench's schedule: both stages of both slots captured as hipGraphs, one half-step
    replayed (A(1) on the side stream beside B(0)), slot 0 compared with the plain step."""
    if pp.graphs_a[0] is None:
        pp.capture()
    for sl, s in zip(pp.slots, s0):
        sl.parts[0].kp.seed.copy_(s)
    pp.reset()
    torch.cuda.synchronize()
    pp.step()
    torch.cuda.synchronize()
    got = bufs(pp.slots[0].parts[0].kp)
    diffs = [k for k in ref if not torch.equal(ref[k], got[k])]
    res = pp.slots[0].results()
    rdiff = [k for k in ref_res if not torch.equal(ref_res[k], res[k])]
    return diffs, rdiff, ""


print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}", flush=True)
for mode in MODES:
    bad = 0
    for r in range(reps):
        diffs, rdiff, detail = trial_graph() if mode == "graph" else trial(mode)
        if diffs or rdiff:
            bad += 1
            print(f"  {mode} rep {r}: buffers {diffs[:8]} results {rdiff}{detail}", flush=True)
    print(f"{mode}: {bad}/{reps} mismatching", flush=True)
