"""hipGraph capture of cross-stream dependencies without events between side streams.

profiles/hip_capture_crosswait.py segfaults at capture end on this image (ROCm 7.2 runtime,
PyTorch 2.10+rocm7.0) whether or not its events stay alive (round 6, profiles/r6_capture_crosswait.txt):
side streams waiting on events recorded on OTHER side streams. The same dependency pattern is
expressed here by hipStreamGetCaptureInfo_v2 (the producer stream's current leaf nodes) +
hipStreamUpdateCaptureDependencies(consumer, nodes, ADD): no event is recorded or waited on
between side streams (only the fork from / join into the origin stream use events, as in every
plan that captures fine). The replayed result is checked against an eager run.

usage (GPU box): python3 profiles/hip_capture_deps.py MODE      MODE = deps | events
"""
import ctypes
import sys

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "deps"
dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipStreamGetCaptureInfo_v2.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.POINTER(ctypes.c_void_p)),
                                           ctypes.POINTER(ctypes.c_size_t)]
hip.hipStreamUpdateCaptureDependencies.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                                   ctypes.c_uint]


def add_deps(src: torch.cuda.Stream, dst: torch.cuda.Stream):
    """dst's next captured work depends on everything captured on src so far."""
    st, cid, graph = ctypes.c_int(), ctypes.c_ulonglong(), ctypes.c_void_p()
    deps, n = ctypes.POINTER(ctypes.c_void_p)(), ctypes.c_size_t()
    e = hip.hipStreamGetCaptureInfo_v2(ctypes.c_void_p(src.cuda_stream), ctypes.byref(st), ctypes.byref(cid),
                                       ctypes.byref(graph), ctypes.byref(deps), ctypes.byref(n))
    assert e == 0 and st.value == 1, (e, st.value)
    nodes = (ctypes.c_void_p * max(1, n.value))(*[deps[k] for k in range(n.value)])
    e = hip.hipStreamUpdateCaptureDependencies(ctypes.c_void_p(dst.cuda_stream), nodes, n.value, 0)  # ADD
    assert e == 0, e


n = 4
xs = [torch.zeros(1 << 18, device=dev) for _ in range(n)]
ys = [torch.zeros(1 << 18, device=dev) for _ in range(n)]
side = [torch.cuda.Stream() for _ in range(n - 1)]
alive = []


def body(main, capture):
    streams = [main] + side
    e0 = torch.cuda.Event()
    alive.append(e0)
    e0.record(main)
    for s in side:
        s.wait_event(e0)
    for j in range(n):
        with torch.cuda.stream(streams[j]):
            xs[j].add_(1)
            xs[j].mul_(1.0001)
    for i in range(n):
        for j in range(n):
            if j != i:
                if capture and mode == "deps":
                    add_deps(streams[j], streams[i])
                else:
                    e = torch.cuda.Event()
                    alive.append(e)
                    e.record(streams[j])
                    streams[i].wait_event(e)
    for i in range(n):
        with torch.cuda.stream(streams[i]):
            ys[i].copy_(xs[i])
            for j in range(n):
                if j != i:
                    ys[i].add_(xs[j], alpha=0.5)
    for s in side:
        e = torch.cuda.Event()
        alive.append(e)
        e.record(s)
        main.wait_event(e)


print("mode", mode, flush=True)
body(torch.cuda.current_stream(), capture=False)
torch.cuda.synchronize()
ref = [y.clone() for y in ys]
for x in xs + ys:
    x.zero_()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body(torch.cuda.current_stream(), capture=True)
print("captured", flush=True)
for x in xs + ys:
    x.zero_()
g.replay()
torch.cuda.synchronize()
ok = all(torch.equal(a, b) for a, b in zip(ys, ref)) and float(ref[0][0]) != 0.0
print("replay ok, equal to eager:", ok, flush=True)
sys.exit(0 if ok else 3)
