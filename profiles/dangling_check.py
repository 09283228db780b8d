"""Use-after-free detector for launch plans: every device pointer baked into a plan op must lie
inside a live CUDA tensor (plan buffers, folded weights, model parameters). A pointer into freed
memory would read / write whatever the caching allocator hands out next, which makes results
depend on what the process allocated before. usage: python3 profiles/dangling_check.py [split]"""
import ctypes
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.runtime import ConvDesc, Op  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

dev = torch.device("cuda", 0)
B, S, N = 4, 64, 256
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=22)
pipes = [BatchPipeline(m, B, S, N, dev, parts=1, seed=0), PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")]
gc.collect()
torch.cuda.synchronize()
ranges = []
for o in gc.get_objects():
    try:
        if isinstance(o, torch.Tensor) and o.is_cuda:
            st = o.untyped_storage()
            ranges.append((st.data_ptr(), st.data_ptr() + st.nbytes()))
    except Exception:
        pass
ranges.sort()
starts = [r[0] for r in ranges]
import bisect  # noqa: E402


def live(p):
    i = bisect.bisect_right(starts, p) - 1
    return i >= 0 and ranges[i][0] <= p < ranges[i][1]


def plans_of(pp):
    if isinstance(pp, BatchPipeline):
        return [(f"part{i}", x) for i, pt in enumerate(pp.parts) for x in (pt.kp.device_perm_plan, pt.kp.plan, pt.pose)]
    return [(f"slot{s}", x) for s, sl in enumerate(pp.slots) for pt in sl.parts for x in
            (pt.kp.device_perm_plan, pt.kp.plan, pt.pose)]


bad = 0
seen = 0
for name, pp in (("plain", pipes[0]), ("pipelined", pipes[1])):
    for tag, plan in plans_of(pp):
        for op in plan.ops:
            if not isinstance(op, Op):
                continue
            ptrs = list(enumerate(op.args))
            if op.name in ("krrn_conv2d_group_x3_f32", "krrn_conv2d_group_f32"):
                n = op.args[1]
                descs = ctypes.cast(ctypes.c_void_p(op.args[0].value), ctypes.POINTER(ConvDesc * n)).contents
                ptrs = [(f"desc{q}.{f}", ctypes.c_void_p(getattr(descs[q], f))) for q in range(n)
                        for f in ("in_", "wt", "scale", "bias", "bias2", "res", "out", "workspace")]
            elif op.name == "krrn_blas_gemm_run":
                ptrs = ptrs[1:]  # arg 0 is the host-side plan handle
            for ai, a in ptrs:
                if isinstance(a, ctypes.c_void_p) and a.value and a.value >= (0x7 << 44):
                    seen += 1
                    if not live(a.value):
                        bad += 1
                        print(f"DANGLING {name}/{tag}: {op.name} arg {ai} = {a.value:#x} meta={op.meta.get('tag')}",
                              flush=True)
print(f"{seen} device pointers checked against {len(ranges)} live tensors: {bad} dangling", flush=True)
