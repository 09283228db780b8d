"""Does stage A (backbone + heads graph of one slot) overlap stage B (fusion / TBase / PnP graph of
the other slot) when the two hipGraphs are replayed on two streams? Times A alone, B alone, A then
B on one stream, and A || B on two streams (the PipelinedPipeline half-step).

usage (GPU box): python3 profiles/overlap_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.pipeline import PipelinedPipeline  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

dev = torch.device("cuda", 0)
B, S, N = 64, 120, 1000
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
pl = PipelinedPipeline(m, B, S, N, dev, seed=3, split=os.environ.get("SPLIT", "heads"))
pl.load(make_batch(B, S, N, seed=1))
pl.capture()
ga, gb = pl.graphs_a, pl.graphs_b
side = torch.cuda.Stream(dev)
main = torch.cuda.current_stream(dev)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def both():
    side.wait_stream(main)
    with torch.cuda.stream(side):
        ga[1].replay()
    gb[0].replay()
    main.wait_stream(side)


print(f"A alone      {timeit(lambda: ga[1].replay()):7.3f} ms", flush=True)
print(f"B alone      {timeit(lambda: gb[0].replay()):7.3f} ms", flush=True)
print(f"A then B     {timeit(lambda: (ga[1].replay(), gb[0].replay())):7.3f} ms", flush=True)
print(f"A || B       {timeit(both):7.3f} ms", flush=True)
