"""End-to-end eval throughput: evaluate.test_epoch over a synthetic LineMOD-all
set — f2 (on-GPU crop / point construction from full 640x480 RGB-D frames), f3 (crops bucketed
by their snapped square size, drawn from LM_CROP_HIST), the KRRN forward (HRNet-W18, 13 classes),
get_pose (PnP-RANSAC on the GPU) and the ADD(-S) metric, per batch of <= 64 — timed over a
whole epoch (best of 3) after a warm-up epoch that builds every (B, S) launch plan.

Reference: tools/trainer.py:145-250 (test_epoch), :521-551 (process_patch_datas),
dataset/linemod/batchdataset.py:603-771 (_load_data).

Prints one JSON line; also times the forward alone over the same batches (inputs prebuilt) so
the loader + pose + metric share of the epoch is visible.

usage (GPU box): python3 profiles/eval_epoch.py [--frames 1024] [--bs 64] [--out FILE]"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("KRRN_PLAN_BUDGET_GB", "200")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config  # noqa: E402
from pose_estimation_amd import distributed as kd  # noqa: E402
from pose_estimation_amd.dataset import PoseDataset  # noqa: E402
from pose_estimation_amd.evaluate import _batches, test_epoch  # noqa: E402
from pose_estimation_amd.synthetic import init_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t = time.time()
    ds = PoseDataset("test", 1000, False, None, 0.0, 8, cls_type="all", num_frames=args.frames, seed=0)
    print(f"synthetic frames: {args.frames} in {time.time() - t:.1f} s", flush=True)
    sizes = [ds.crop_size(i) for i in range(len(ds))]
    hist = {s: sizes.count(s) for s in sorted(set(sizes))}
    m = KRRN(cfg=make_config(num_cls=len(ds.objlist), backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    t = time.time()
    test_epoch(m, ds, bs=args.bs, device=dev)  # warm-up: one launch plan per (B, S)
    torch.cuda.synchronize()
    print(f"warm-up epoch (plan builds) {time.time() - t:.1f} s", flush=True)
    times = []
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.time()
        res = test_epoch(m, ds, bs=args.bs, device=dev)
        torch.cuda.synchronize()
        times.append(time.time() - t)
        print(f"epoch {times[-1]:.3f} s", flush=True)
    assert res["test_count"] == len(ds)
    ep = min(times)
    # the forward alone over the same batches, inputs prebuilt
    buckets = kd.bucket_shard(sizes, 1, 0)
    batches = [ds.batch(idx, dev) for _, idx in _batches(buckets, args.bs)]
    with torch.no_grad():
        for d in batches:
            m(d["img_croped"], d["cloud"], d["choose"], d["cls_id"])
        torch.cuda.synchronize()
        fwds = []
        for _ in range(3):  # best of 3, like the epoch
            t = time.time()
            for d in batches:
                m(d["img_croped"], d["cloud"], d["choose"], d["cls_id"])
            torch.cuda.synchronize()
            fwds.append(time.time() - t)
        fwd = min(fwds)
    line = {"metric": "eval crops/s, evaluate.test_epoch end to end (f2 inputs + forward + get_pose + ADD(-S))",
            "value": round(len(ds) / ep, 2), "unit": "crops/s", "epoch_s": round(ep, 4), "crops": len(ds),
            "batches": len(batches), "bs": args.bs, "size_hist": hist, "forward_only_s": round(fwd, 4),
            "forward_only_crops_s": round(len(ds) / fwd, 2), "classes": len(ds.objlist),
            "data": "synthetic LineMOD-all frames (640x480 RGB-D, LM_CROP_HIST sizes), random-init HRNet-W18 KRRN",
            "n_gpus": 1}
    print(json.dumps(line), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
