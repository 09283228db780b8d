"""BPnP timing: krrn_bpnp_solve_f32 (LM forward from a perturbed guess) and
krrn_bpnp_backward_f32 on MI355X at B crops x n points, beside the CPU oracle's autograd
backward (the reference algorithm, oracle/bpnp_oracle.py) on a bounded sample of crops.

usage (GPU box): python3 profiles/bench_bpnp.py [out.json]   (env B, N)
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import bpnp_oracle as bo  # noqa: E402  (CPU baseline only)
from pose_estimation_amd import bpnp  # noqa: E402

B, N = int(os.environ.get("B", 64)), int(os.environ.get("N", 256))
dev = torch.device("cuda", 0)
K = np.array([[572.4114, 0, 325.2611], [0, 573.57043, 242.04899], [0, 0, 1]])
rng = np.random.default_rng(0)
z = (rng.random((N, 3)) - 0.5) * 0.15
ys, xs = [], []
for _ in range(B):
    w = rng.normal(size=3)
    w *= rng.uniform(0.3, 2.5) / np.linalg.norm(w)
    y = np.concatenate([w, [rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.6, 1.1)]])
    ys.append(y)
    xs.append(bo._residual(y, np.zeros((N, 2)), z, K).reshape(N, 2) + 0.5 * rng.normal(size=(N, 2)))
y = np.stack(ys)
y0 = y + np.concatenate([rng.normal(size=(B, 3)) * 0.05, rng.normal(size=(B, 3)) * 0.01], axis=1)
f = lambda a: torch.tensor(np.asarray(a, np.float32), device=dev)  # noqa: E731
x_t, z_t, K_t, y0_t = f(np.stack(xs)), f(z), f(K), f(y0)
g_t = f(rng.normal(size=(B, 6)))


def ev_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


P6 = bpnp.solve(x_t, z_t, K_t, ini_pose=y0_t)
t_solve = ev_time(lambda: bpnp.solve(x_t, z_t, K_t, ini_pose=y0_t))
t_bwd = ev_time(lambda: bpnp.backward(x_t, P6, z_t, K_t, g_t))
torch.set_num_threads(min(16, os.cpu_count() or 1))
nc, t0 = 0, time.perf_counter()
P6c = P6.cpu().numpy()
while time.perf_counter() - t0 < 10.0 and nc < B:
    bo.bpnp_backward(np.stack(xs)[nc:nc + 1].astype(np.float32), P6c[nc:nc + 1], z.astype(np.float32),
                     K.astype(np.float32), g_t.cpu().numpy()[nc:nc + 1])
    nc += 1
cpu_s = (time.perf_counter() - t0) / nc
res = {"B": B, "n": N, "solve_ms": round(t_solve, 4), "backward_ms": round(t_bwd, 4),
       "backward_crops_per_s": round(B / (t_bwd / 1e3), 1), "solve_crops_per_s": round(B / (t_solve / 1e3), 1),
       "cpu_oracle_backward_crops_per_s": round(1.0 / cpu_s, 2), "cpu_threads": torch.get_num_threads(),
       "cpu_sample": f"{nc} crops of the same workload, oracle/bpnp_oracle.py (torch autograd, f32)",
       "note": "latency-bound (one wave per crop, f64); reported absolute, not against a roofline"}
print(json.dumps(res))
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
