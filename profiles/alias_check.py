"""Cross-plan aliasing detector: every device pointer baked into a plan's launches must lie in memory
that plan (or the model) owns. A pointer that lands inside ANOTHER plan's buffer is a use-after-free
whose memory the caching allocator handed to that plan: its kernel then reads / writes the other
plan's data, and with the two plans running concurrently (PipelinedPipeline) the result depends on
timing. Builds the same sequence as tests/test_gpu_pipeline.py::test_pipelined_graph_benched_shape
(with HISTORY=1 the other pipeline tests first) and reports every such pointer.

usage (GPU box): [HISTORY=1] python3 profiles/alias_check.py [B S N]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.runtime import ConvDesc, Op  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

dev = torch.device("cuda", 0)
if os.environ.get("HISTORY"):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    import test_gpu_pipeline as tgp  # noqa: E402
    for name, args in (("test_pipeline_matches_api_and_graph", (1,)), ("test_pipeline_matches_api_and_graph", (2,)),
                       ("test_pipelined_matches_plain", ("heads",))):
        try:
            getattr(tgp, name)(dev, *args)
        except AssertionError:
            pass
B, S, N = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 120, 1000)
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=1)
plain = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
plain.load(d)
plain.run()
torch.cuda.synchronize()
del plain
pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")
pp.load(d)
torch.cuda.synchronize()


def tensors(obj, out, depth=0):
    """Every CUDA tensor reachable from a plan's buffers / keep lists."""
    if depth > 6:
        return
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for x in obj:
            tensors(x, out, depth + 1)
    elif isinstance(obj, dict):
        for x in obj.values():
            tensors(x, out, depth + 1)
    elif hasattr(obj, "__dict__"):
        for x in vars(obj).values():
            tensors(x, out, depth + 1)


def ranges_of(ts):
    r = []
    for t in ts:
        st = t.untyped_storage()
        r.append((st.data_ptr(), st.data_ptr() + st.nbytes()))
    return r


def pointers(op):
    out = []
    for ai, a in enumerate(op.args):
        if op.name == "krrn_blas_gemm_run" and ai == 0:
            continue
        if isinstance(a, ctypes.c_void_p) and a.value:
            out.append((str(ai), a.value))
        elif isinstance(a, ctypes.Array):
            for k, v in enumerate(a):
                if isinstance(v, int) and v > (1 << 40):
                    out.append((f"{ai}[{k}]", v))
    if op.name in ("krrn_conv2d_group_x3_f32", "krrn_conv2d_group_f32"):
        st = ConvDesc
        n = op.args[1]
        descs = ctypes.cast(ctypes.c_void_p(op.args[0].value), ctypes.POINTER(st * n)).contents
        for q in range(n):
            for f, ft in st._fields_:
                if ft is ctypes.c_void_p:
                    v = getattr(descs[q], f)
                    if v:
                        out.append((f"desc{q}.{f}", v))
    return out


owners = []  # (name, plan, ranges)
for s, sl in enumerate(pp.slots):
    pt = sl.parts[0]
    for pname, plan in (("perm", pt.kp.device_perm_plan), ("plan", pt.kp.plan), ("pose", pt.pose)):
        ts = []
        tensors(plan.buffers, ts)
        tensors([pt.kp, pt], ts)
        owners.append((f"slot{s}/{pname}", plan, ranges_of(ts)))
model_ranges = ranges_of([p for p in m.parameters()] + [b for b in m.buffers()])
slot_ranges = {}
for name, plan, rs in owners:
    slot_ranges.setdefault(name.split("/")[0], []).extend(rs)


def inside(p, rs):
    return any(lo <= p < hi for lo, hi in rs)


bad = seen = 0
for name, plan, _ in owners:
    mine = slot_ranges[name.split("/")[0]]
    others = {k: v for k, v in slot_ranges.items() if k != name.split("/")[0]}
    for oi, op in enumerate(plan.ops):
        if not isinstance(op, Op):
            continue
        for tag, p in pointers(op):
            seen += 1
            if inside(p, mine) or inside(p, model_ranges):
                continue
            hit = [k for k, v in others.items() if inside(p, v)]
            bad += 1
            print(f"{'ALIAS' if hit else 'UNOWNED'} {name} op {oi} {op.name} arg {tag} = {p:#x} "
                  f"{'-> inside ' + ','.join(hit) if hit else ''} meta={op.meta.get('tag') if op.meta else None}",
                  flush=True)
print(f"{seen} pointers checked: {bad} not owned by their slot (or the model)", flush=True)
