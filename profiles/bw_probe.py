"""HBM bandwidth probe: what torch's own streaming kernels reach on this box for write-only (fill),
read + write (copy) and read-only (sum) traffic at the sizes of the step's big launches. It gives
the practical ceiling that the write-heavy kernels (the K = 128 GCN GEMMs, resize_up2x2) are
judged against.

usage (GPU box): python3 profiles/bw_probe.py [MB ...]"""
import json
import sys

import torch

sizes = [int(v) for v in sys.argv[1:]] or [256, 512, 1024]
dev = torch.device("cuda", 0)
out = {}
for mb in sizes:
    n = mb * (1 << 20) // 4
    a = torch.empty(n, device=dev)
    b = torch.empty(n, device=dev)
    a.fill_(1.0)
    res = {}
    for name, fn, nbytes in (("fill", lambda: b.fill_(2.0), 4 * n), ("copy", lambda: b.copy_(a), 8 * n),
                             ("sum", lambda: a.sum(), 4 * n)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[name] = {"us": round(us, 1), "TB/s": round(nbytes / us / 1e6, 2)}
    out[f"{mb}MB"] = res
    print(mb, res, flush=True)
print(json.dumps(out))
