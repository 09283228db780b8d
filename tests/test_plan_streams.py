"""The forward plan's stream structure, checked on a CPU build (no GPU): the rules a hipGraph capture
of it has to satisfy. A side stream may run work only after it waited on an event of a stream that
is already in the capture (a fork), and every side stream's work must be joined back into stream 0
before the capture ends. The pipeline's stage graphs (runtime.Plan slices at KRRNPlan.split /
heads_end) need the same at their cut points. A plan that breaks these fails at capture on the GPU
(or, worse, replays with a missing edge)."""
import torch

from pose_estimation_amd import KRRN, make_config
from pose_estimation_amd.krrn import KRRNPlan
from pose_estimation_amd.runtime import Sync
from pose_estimation_amd.synthetic import init_weights


def _check(ops):
    """Simulate capture over `ops`; returns (problems, side streams with unjoined work)."""
    capturing, pending, problems = {0}, {}, []
    for k, op in enumerate(ops):
        if isinstance(op, Sync):
            if op.src not in capturing:
                problems.append((k, "wait on a stream outside the capture", op.src, op.dst))
            capturing.add(op.dst)
            if op.dst == 0:
                pending.pop(op.src, None)
            continue
        if op.sid not in capturing:
            problems.append((k, "launch on a stream outside the capture", op.sid, op.name))
        if op.sid != 0:
            pending[op.sid] = k
    return problems, pending


def test_forward_plan_streams_fork_and_join():
    torch.manual_seed(0)
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m.eval()
    kp = KRRNPlan(m, 2, 64, 256, True, torch.device("cpu"))
    ops = kp.plan.ops
    assert kp.plan.nstreams > 4  # HRNet branches, heads and fusion branches on side streams
    for name, cut in (("backbone", kp.split), ("heads", kp.heads_end), ("whole plan", len(ops))):
        problems, pending = _check(ops[:cut])
        assert not problems, (name, problems[:5])
        assert not pending, (name, "side streams not joined", pending)
    # the stage after each cut starts from a joined state too
    for cut in (kp.split, kp.heads_end):
        problems, pending = _check(ops[cut:])
        assert not problems and not pending, (cut, problems[:5], pending)
