"""Diagnostic: the bench's step (BatchPipeline: device draws + forward with get_pose on its own stream
+ rng advance) run serially vs captured with its side streams into a hipGraph and replayed, REPS
times, alternating between two RNG states so that a kernel reading a buffer before this step's
producer wrote it sees the OTHER state's values (identical replays would hide such a race); with
PIPE=heads the PipelinedPipeline half-step graphs instead. Prints every plan buffer that differs
from the serial run of the same state, in allocation order, with the first op (index, name,
stream) that touches it.

usage (GPU box): REPS=5 [PIPE=heads] python3 profiles/pipe_vs_graph.py [B S N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.runtime import Op  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

B, S, N = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 120, 1000)
REPS = int(os.environ.get("REPS", "5"))
PIPE = os.environ.get("PIPE", "")
dev = torch.device("cuda", 0)
if os.environ.get("HISTORY"):
    # the history under which tests/test_gpu_pipeline.py mismatched: its other tests first
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    import test_gpu_pipeline as tgp  # noqa: E402
    for name, args in (("test_pipeline_matches_api_and_graph", (1,)), ("test_pipeline_matches_api_and_graph", (2,)),
                       ("test_pipelined_matches_plain", ("heads",))):
        try:
            getattr(tgp, name)(dev, *args)
        except AssertionError:
            print(f"history {name}{args}: mismatch", flush=True)
INNER = os.environ.get("INNER", "1") == "1"  # 0: the graph captured on one stream (no plan side streams)
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=9)


def buffers_of(pl):
    out, first = [], {}
    for plan, _ in pl.plans():
        ts = [t for t in plan.buffers if isinstance(t, torch.Tensor)]
        for oi, op in enumerate(plan.ops):
            if not isinstance(op, Op):
                continue
            for a in op.args:
                v = getattr(a, "value", None)
                if not v:
                    continue
                for t in ts:
                    lo = t.data_ptr()
                    if lo <= v < lo + t.numel() * t.element_size() and lo not in first:
                        first[lo] = (oi, op.name, op.sid)
        out += ts
    return out, first


def report(tag, ref, cur, bufs, first):
    bad = [i for i in range(len(bufs)) if not torch.equal(ref[i], cur[i])]
    print(f"{tag}: {len(bad)} buffers differ", flush=True)
    for i in bad[:10]:
        a, b = ref[i], cur[i]
        diff = float((a.double() - b.double()).abs().max()) if a.is_floating_point() else int((a != b).sum())
        print(f"   buf {i} {tuple(a.shape)} {a.dtype} first op {first.get(bufs[i].data_ptr())} maxdiff {diff:.3e}",
              flush=True)


if not PIPE:
    pl = BatchPipeline(m, B, S, N, dev, parts=1, seed=3, inner_streams=INNER)
    pl.load(d)
    bufs, first = buffers_of(pl)
    seeds = [pl.parts[0].kp.seed.clone(), pl.parts[0].kp.seed.clone() + 12345]
    refs = []
    for sd in seeds:
        pl.parts[0].kp.seed.copy_(sd)
        pl.run()
        torch.cuda.synchronize()
        refs.append([t.clone() for t in bufs])
    pl.capture()
    for r in range(REPS):
        pl.parts[0].kp.seed.copy_(seeds[r % 2])
        pl.step()
        torch.cuda.synchronize()
        report(f"graph replay {r} (state {r % 2})", refs[r % 2], [t.clone() for t in bufs], bufs, first)
else:
    plain = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
    plain.load(d)
    sp = plain.parts[0].kp.seed.clone()
    wants = []
    for off in (0, 12345):
        plain.parts[0].kp.seed.copy_(sp + off)
        plain.run()
        torch.cuda.synchronize()
        wants.append({k: v.clone() for k, v in plain.results().items()})
    pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split=PIPE)
    pp.load(d)
    s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]
    pp.capture()
    for r in range(REPS):
        off = 12345 * (r % 2)
        for sl, s in zip(pp.slots, s0):
            sl.parts[0].kp.seed.copy_(s + off)
        pp.reset()
        pp.step()
        torch.cuda.synchronize()
        got = pp.results()
        bad = [k for k in wants[r % 2] if not torch.equal(got[k], wants[r % 2][k])]
        print(f"pipelined replay {r} (state {r % 2}): differs in {bad}", flush=True)
