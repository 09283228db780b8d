"""Micro-bench: krrn_knn_f32 on the fusion's shapes (B = 64, N = 1000), 4 vs 16 lanes per query
(the lanes-per-query rule is fixed in gcn.hip since round 5: build a variant library with the other
choice and point KRRN_HIP_LIB at it, profiles/build_variant.sh); prints a checksum of the indices
so both runs can be compared for equality. The "pixel-ordered" cases use crops like the step's:
1000 mask pixels of a 48 x 48 window in raster order (choose), back-projected from a smooth depth."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

dev = torch.device("cuda", 0)
B, N = 64, 1000
g = torch.Generator().manual_seed(0)
pts = torch.rand(B, N, 9, generator=g).to(dev)
perm = torch.randperm(N, generator=g)[:250].int().to(dev)
# pixel-ordered crops: raster-order mask pixels of a 48 x 48 window, back-projected
u, v = torch.meshgrid(torch.arange(48.0), torch.arange(48.0), indexing="xy")
inside = ((u - 23.5) / 24) ** 2 + ((v - 23.5) / 22) ** 2 < 1.0
pix = torch.nonzero(inside.flatten()).flatten()
crops = []
for bb in range(B):
    sel = pix[torch.randperm(len(pix), generator=g)[:N]].sort().values
    uu, vv = u.flatten()[sel], v.flatten()[sel]
    z = 0.6 + 0.05 * torch.sin(uu / 7 + bb) + 0.03 * torch.cos(vv / 5) + 0.002 * torch.rand(N, generator=g)
    rec = torch.zeros(N, 9)
    rec[:, 0], rec[:, 1], rec[:, 2] = (uu - 24) * z / 570, (vv - 24) * z / 570, z
    rec[:, 3:] = torch.rand(N, 6, generator=g)
    crops.append(rec)
ordered = torch.stack(crops).to(dev)
st = P(torch.cuda.current_stream().cuda_stream)
# (name, nq, qidx, nc, d, k, drop, mode)
cases = [("level0 pixel-ordered", 1000, None, 1000, 3, 10, 1, 0, ordered),
         ("level0 idx0", 1000, None, 1000, 3, 10, 1, 0), ("pool k4", 250, perm, 1000, 3, 4, 1, 0),
         ("level1 idx1", 250, None, 250, 3, 10, 1, 0), ("level2 idx2 9-D", 62, None, 62, 9, 7, 1, 0),
         ("nn1", 1000, None, 250, 3, 1, 0, 1), ("nn2", 1000, None, 62, 3, 1, 0, 1)]
for name, nq, qidx, nc, d, k, drop, mode, *src in cases:
    src = src[0] if src else pts
    out = torch.zeros(B, nq, k, dtype=torch.int32, device=dev)
    fn = lambda: _lib.check(_lib.lib().krrn_knn_f32(ptr(src), N * 9, 9, nq, ptr(qidx), ptr(src), N * 9, 9, nc, d, k,  # noqa: E731
                                                    drop, mode, B, ptr(out), st), "knn")
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    cs = int((out.long() * torch.arange(out.numel(), device=dev).view_as(out).remainder(9973)).sum())
    print(f"{name:18s} {a.elapsed_time(b) / 20 * 1e3:8.1f} us  checksum {cs}", flush=True)
