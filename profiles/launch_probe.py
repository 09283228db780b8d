"""Per-launch cost of a dependent chain of tiny kernels inside a hipGraph (what bounds a plan of
~430 short launches): 200 one-block launches on one stream, and 4 x 50 on four forked streams.

usage (GPU box): python3 profiles/launch_probe.py
"""
import torch

dev = torch.device("cuda", 0)
x = torch.zeros(64, device=dev)
xs = [torch.zeros(64, device=dev) for _ in range(4)]


def chain(n, t):
    for _ in range(n):
        t.add_(1.0)


def forked(n):
    cur = torch.cuda.current_stream(dev)
    ss = [torch.cuda.Stream(dev) for _ in range(3)]
    for s in ss:
        s.wait_stream(cur)
    chain(n, xs[0])
    for s, t in zip(ss, xs[1:]):
        with torch.cuda.stream(s):
            chain(n, t)
    for s in ss:
        cur.wait_stream(s)


def graph_time(fn, reps=20):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


t1 = graph_time(lambda: chain(200, x))
print(f"200 dependent launches, 1 stream : {t1 * 1e3 / 200:6.2f} us per launch", flush=True)
t4 = graph_time(lambda: forked(50))
print(f"4 x 50 launches on 4 streams     : {t4 * 1e3 / 50:6.2f} us per 4-wide step", flush=True)
