"""Repro (plain PyTorch, no KRRN code): hipGraph capture segfaults at capture end on this image
(ROCm 7.2 runtime, PyTorch 2.10+rocm7.0) when each of 4 streams records several events at
different points and every stream then waits on the others' events. Found while giving each HRNet
fuse output a wait on exactly the terms it needs; the plan keeps the
module-level barrier instead. Not run by any test.

usage (GPU box, expect rc 139): python3 profiles/hip_capture_crosswait.py 1
"""
import torch, sys
dev = torch.device('cuda', 0)
n = 4
xs = [torch.zeros(1 << 18, device=dev) for _ in range(n)]
pre = {}
side = [torch.cuda.Stream() for _ in range(n - 1)]
def body(main):
    streams = [main] + side
    e0 = torch.cuda.Event(); e0.record(main)
    for s in side: s.wait_event(e0)
    marks = {}
    for j in range(n):
        with torch.cuda.stream(streams[j]):
            xs[j].add_(1)
            for i in range(n):
                if i != j:
                    xs[j].mul_(1.0001)
                    e = torch.cuda.Event(); e.record(streams[j]); marks[(i, j)] = e
    outs = []
    for i in range(n):
        for j in range(n):
            if j != i:
                streams[i].wait_event(marks[(i, j)])
                with torch.cuda.stream(streams[i]): xs[i].add_(xs[j])
    for s in side:
        e = torch.cuda.Event(); e.record(s); main.wait_event(e)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for rep in range(int(sys.argv[1])):
        body(torch.cuda.current_stream())
print("captured", flush=True)
g.replay(); torch.cuda.synchronize(); print("replay ok", flush=True)
