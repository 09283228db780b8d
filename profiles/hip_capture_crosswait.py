"""Repro (plain PyTorch, no KRRN code) of the hipGraph capture segfault seen in round 5 when each
HRNet fuse output waited on exactly the terms it needs. Each of 4 streams
records several events at different points and every stream then waits on the others' events.

usage (GPU box): python3 profiles/hip_capture_crosswait.py REPS [keep]
  keep   every torch.cuda.Event created inside the capture is kept alive until after
         capture_end (a module-level list); without it, events made in body() are destroyed
         (hipEventDestroy) while the capture is still open: the `marks` dict at body's return, and
         the join loop's `e` each time the name is rebound.
Round 6 runs both forms once (profiles/r6_capture_crosswait.txt). Not run by any test.
"""
import sys

import torch

dev = torch.device('cuda', 0)
n = 4
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
KEEP = len(sys.argv) > 2 and sys.argv[2] == "keep"
alive = []  # events kept until after capture_end (KEEP)
xs = [torch.zeros(1 << 18, device=dev) for _ in range(n)]
side = [torch.cuda.Stream() for _ in range(n - 1)]


def event():
    e = torch.cuda.Event()
    if KEEP:
        alive.append(e)
    return e


def body(main):
    streams = [main] + side
    e0 = event()
    e0.record(main)
    for s in side:
        s.wait_event(e0)
    marks = {}
    for j in range(n):
        with torch.cuda.stream(streams[j]):
            xs[j].add_(1)
            for i in range(n):
                if i != j:
                    xs[j].mul_(1.0001)
                    e = event()
                    e.record(streams[j])
                    marks[(i, j)] = e
    for i in range(n):
        for j in range(n):
            if j != i:
                streams[i].wait_event(marks[(i, j)])
                with torch.cuda.stream(streams[i]):
                    xs[i].add_(xs[j])
    for s in side:
        e = event()
        e.record(s)
        main.wait_event(e)


print(f"reps {reps} keep {KEEP}", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for rep in range(reps):
        body(torch.cuda.current_stream())
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", float(xs[0][0]), flush=True)
