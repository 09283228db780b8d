"""Diagnostic: first buffer where PipelinedPipeline(split) differs from the plain BatchPipeline
(same seed), optionally after other GPU tests ran in the same process.
usage: python3 profiles/diag_pipeline.py [split | plain] [pytest files to run first ...]"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
split = sys.argv[1] if len(sys.argv) > 1 else "heads"
if len(sys.argv) > 2:
    pytest.main(["-q", "-p", "no:cacheprovider"] + sys.argv[2:])
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

dev = torch.device("cuda", 0)
B, S, N = 4, 64, 256
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
d = make_batch(B, S, N, seed=22)


def bufs(kp):
    out = {"xyz": kp.xyz, "normal": kp.normal, "fx": kp.fx, "fn": kp.fn, "p9": kp.p9, "pred_t": kp.pred_t}
    out.update({f"perm_{k}": v for k, v in kp.perms.items()})
    for k, v in kp.fusion_bufs.items():
        for i, t in enumerate(v if isinstance(v, list) else [v]):
            if isinstance(t, torch.Tensor):
                out[f"fus_{k}" + (f"[{i}]" if isinstance(v, list) else "")] = t
    out.update({f"tb_{k}": v for k, v in kp.tbase_bufs.items() if isinstance(v, torch.Tensor)})
    return {k: v.clone() for k, v in out.items()}


plain = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
plain.load(d)
plain.run()
torch.cuda.synchronize()
ref = bufs(plain.parts[0].kp)
if split == "plain":  # a second plain pipeline: run-to-run / plan-to-plan determinism
    pp = BatchPipeline(m, B, S, N, dev, parts=1, seed=0)
    pp.load(d)
    pp.run()
    torch.cuda.synchronize()
    got = bufs(pp.parts[0].kp)
else:
    pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split=split)
    pp.load(d)
    pp.run()
    torch.cuda.synchronize()
    got = bufs(pp.slots[0].parts[0].kp)
for k in ref:
    a, b = ref[k], got[k]
    same = torch.equal(a, b)
    diff = 0.0 if same else float((a.double() - b.double()).abs().max())
    print(f"{k:24s} {'same' if same else 'DIFF'} {diff:.3e} {tuple(a.shape)}", flush=True)
a, b = ref["fus_feat2"], got["fus_feat2"]
for bi in range(3):
    sl = slice(128 * bi, 128 * bi + 128)
    dd = (a[..., sl] - b[..., sl]).abs().amax(-1)  # [B, N1]
    print(f"feat2 slice {bi}: max {float(dd.max()):.3e}, rows differing {int((dd > 0).sum())} of {dd.numel()}",
          flush=True)
