"""Which launch forms run concurrently on this runtime? A spin kernel (torch.cuda._sleep, one
block) of ~T ms issued twice: eagerly on two streams, as two graphs replayed on two streams, and as
one graph whose capture forks into two streams. ~T = concurrent, ~2T = serialised.

usage (GPU box): python3 profiles/concurrency_probe.py
"""
import torch

dev = torch.device("cuda", 0)
CYC = 20_000_000
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
main = torch.cuda.current_stream(dev)


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def one():
    torch.cuda._sleep(CYC)


def eager_two():
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(CYC)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(CYC)
    main.wait_stream(s1)
    main.wait_stream(s2)


def capture(fn):
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    cs.wait_stream(main)
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g, stream=cs):
            fn()
    main.wait_stream(cs)
    torch.cuda.synchronize()
    return g


g1, g2 = capture(one), capture(one)


def graphs_two():
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        g1.replay()
    with torch.cuda.stream(s2):
        g2.replay()
    main.wait_stream(s1)
    main.wait_stream(s2)


def forked():
    cur = torch.cuda.current_stream(dev)
    f = torch.cuda.Stream(dev)
    f.wait_stream(cur)
    torch.cuda._sleep(CYC)
    with torch.cuda.stream(f):
        torch.cuda._sleep(CYC)
    cur.wait_stream(f)


gf = capture(forked)
t1 = timeit(one)
print(f"one spin               {t1:7.3f} ms", flush=True)
print(f"eager, two streams     {timeit(eager_two):7.3f} ms", flush=True)
print(f"two graphs, two streams{timeit(graphs_two):7.3f} ms", flush=True)
print(f"one graph, forked      {timeit(lambda: gf.replay()):7.3f} ms", flush=True)
