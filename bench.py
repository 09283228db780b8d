"""KRRN inference benchmark on MI355X (BASELINE.json metric: crops/s).

A step = one pass of the hot path over one batch of synthetic LineMOD crops resident in HBM:
HRNet-W18 + heads + class select/normalise + choose gather + FusionNetLite + TBase (pred_t)
+ batched PnP-RANSAC (R), including the device-side randomness (pool permutations, the 256-
point PnP subset, RANSAC hypotheses). By default the step is a two-stage software pipeline over
two batch slots (pipeline.PipelinedPipeline, split after the heads): stage A = backbone + heads of
batch k+1 and stage B = fusion + TBase + PnP of batch k replay as two hipGraphs on two streams, so
every step completes one whole batch (the latency-bound tail overlaps MFMA-bound convs);
--pipeline none runs one batch end to end as one hipGraph. With --gpus N
(torchrun, one process per GPU, RCCL) every rank runs its own batch (weak scaling) and the
per-crop pose records are all-gathered over RCCL after every step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--size 120] [--points 1000]

Rank 0 prints ONE JSON line (metric, value = crops/s over all ranks, roofline of the dominant
kernel measured with HIP events, cpu_baseline = the CPU oracle on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pose_estimation_amd import distributed as kd  # noqa: E402
from pose_estimation_amd.config import make_config  # noqa: E402
from pose_estimation_amd.krrn import KRRN  # noqa: E402
from pose_estimation_amd.pipeline import BatchPipeline, PipelinedPipeline  # noqa: E402
from pose_estimation_amd.synthetic import OBJ_DICT, init_weights, make_batch  # noqa: E402

METRIC = "crops/sec at 640×480 RGB-D, 1000 sampled pts; ADD(-S) AUC vs reference"
PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32-input MFMA (= f32 vector peak)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


# compulsory fusion HBM bytes per crop (fp32 features, int32 indices; each GCN
# GEMM output written once and read once, every other tensor read or written once)
FUSION_BYTES_PER_CROP = {1000: 49.7e6, 4096: 202.6e6}


def fusion_roofline(prof, fusion_ids, B: int, N: int):
    """FusionNetLite as one unit: algorithmic bytes / serial device time of
    its launches vs the HBM peak (north_star target >= 40 %), and the GCN GEMMs' MFMA rate."""
    ops = [(op, ms) for op, ms in prof if id(op) in fusion_ids]
    if not ops:
        return None
    ms = sum(t for _, t in ops)
    gemm_ms = sum(t for op, t in ops if op.meta.get("flops"))
    gemm_fl = sum(op.meta.get("flops", 0.0) for op, _ in ops)
    per_crop = FUSION_BYTES_PER_CROP.get(N)
    out = {"ms_per_step": round(ms, 3), "launches": len(ops), "gemm_ms": round(gemm_ms, 3),
           "gemm_TFLOP/s": round(gemm_fl / (gemm_ms * 1e-3) / 1e12, 2) if gemm_ms else None}
    if per_crop:
        gbs = per_crop * B / (ms * 1e-3) / 1e9
        out.update({"bound": "hbm", "bytes_per_crop": per_crop, "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4)})
    return out


def roofline_from_profile(prof, B: int):
    groups = {}
    for op, ms in prof:
        k = op.meta.get("kernel", op.name)
        g = groups.setdefault(k, {"ms": 0.0, "flops": 0.0, "mfma": 0.0, "n": 0})
        g["ms"] += ms
        g["flops"] += op.meta.get("flops", 0.0)
        g["mfma"] += op.meta.get("mfma_flops", op.meta.get("flops", 0.0))
        g["n"] += 1
    total_ms = sum(g["ms"] for g in groups.values())
    dom = max(groups, key=lambda k: groups[k]["ms"])
    g = groups[dom]
    avg_ms = g["ms"] / g["n"]
    achieved = (g["flops"] / g["n"]) / (avg_ms * 1e-3) / 1e12 if g["flops"] > 0 else None
    conv_ms = sum(v["ms"] for k, v in groups.items() if k.startswith("conv_gemm"))
    conv_fl = sum(v["flops"] for k, v in groups.items() if k.startswith("conv_gemm"))
    allc = [v for k, v in groups.items() if k.startswith(("conv_gemm", "conv_group", "wino"))]
    allc_ms, allc_fl, allc_mf = (sum(v[f] for v in allc) for f in ("ms", "flops", "mfma"))
    breakdown = {k: {"ms": round(v["ms"], 4), "launches": v["n"],
                     **({"TFLOP/s": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2)} if v["flops"] else {})}
                 for k, v in sorted(groups.items(), key=lambda kv: -kv[1]["ms"])}
    traffic, tsrc = _pmc_traffic(dom)
    roof = {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 2) if achieved else None,
            "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_F32_MFMA_TFLOPS, 4) if achieved else None, "traffic": traffic,
            "traffic_unit": "HBM bytes per launch", "traffic_source": tsrc,
            "launches": g["n"], "avg_launch_us": round(avg_ms * 1e3, 2),
            "flops_per_launch": round(g["flops"] / g["n"]),
            "all_conv_gemm": {"ms_per_step": round(conv_ms, 3),
                              "TFLOP/s": round(conv_fl / (conv_ms * 1e-3) / 1e12, 2) if conv_ms else None,
                              "GFLOP_per_crop": round(conv_fl / B / 1e9, 3)},
            "all_conv": {"ms_per_step": round(allc_ms, 3), "GFLOP_per_crop": round(allc_fl / B / 1e9, 3),
                         "TFLOP/s": round(allc_fl / (allc_ms * 1e-3) / 1e12, 2) if allc_ms else None,
                         "frac": round(allc_fl / (allc_ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4) if allc_ms else None,
                         "mfma_pipe_frac": round(allc_mf / (allc_ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4)
                         if allc_ms else None,
                         "note": "every conv / GEMM of the step incl. Winograd, direct-conv FLOPs (SURVEY §8d)"},
            "events_ms_per_step": round(total_ms, 3)}
    if g["mfma"] and abs(g["mfma"] - g["flops"]) > 1e-6 * g["flops"]:
        # Winograd: `achieved` counts the direct-conv FLOPs the launch replaces (SURVEY §8d's
        # formula), so frac can exceed 1; this is what the matrix pipe actually issued
        mp = (g["mfma"] / g["n"]) / (avg_ms * 1e-3) / 1e12
        roof["mfma_pipe"] = {"achieved": round(mp, 2), "frac": round(mp / PEAK_F32_MFMA_TFLOPS, 4),
                             "flops_per_launch": round(g["mfma"] / g["n"]),
                             "note": "F(2x2,3x3) Winograd issues 2.25x fewer MFMA FLOPs than the direct conv"}
    return roof, breakdown


def _pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of this
    same bench command (profiles/r*_pmc_traffic.json, built by profiles/pmc_traffic.py with the
    gfx950 FETCH_SIZE x2 correction). None when no summary exists."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    if kernel not in d:
        return None, None
    return round(d[kernel]["hbm_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def cpu_baseline(B: int, S: int, N: int, backbone: str, budget_s: float):
    """The CPU oracle (PyTorch-CPU restatement + C EPnP-RANSAC) on a bounded sample."""
    from oracle.krrn_oracle import KRRNOracle, get_pose
    from pose_estimation_amd.fusion import level_sizes
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    m = KRRN(cfg=make_config(num_cls=1, backbone=backbone))
    sd = init_weights(m, 0)
    o = KRRNOracle(num_cls=1, backbone=backbone)
    o.load_state_dict(sd)
    o.eval()
    bcpu = 2
    d = make_batch(bcpu, S, N, seed=99)
    N1, N2, _, _ = level_sizes(N, 10)

    def one():
        perms = [torch.randperm(N)[:N1] for _ in range(4)] + [torch.randperm(N1)[:N2]]
        pred = o(d["img_croped"], d["cloud"], d["choose"], d["cls_id"], perms=perms)
        sel = torch.stack([torch.randperm(N)[:256] for _ in range(bcpu)])
        subs = torch.stack([torch.stack([torch.randperm(256)[:5] for _ in range(100)]) for _ in range(bcpu)])
        get_pose(pred, d, sel, subs.int())
    one()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += bcpu
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": round(n / el, 4), "unit": "crops/s", "cores": threads, "kind": "port",
            "sample": f"{n} crops ({n // bcpu} batches of {bcpu}), S={S}, N={N}, HRNet-{backbone}, oracle/krrn_oracle.py "
                      f"f32 + oracle/pnp_ref.c EPnP-RANSAC H=100, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=120)
    ap.add_argument("--points", type=int, default=1000)
    ap.add_argument("--backbone", default="w18")
    ap.add_argument("--classes", type=int, default=1,
                    help="NUM_CLS (1 = LineMOD 'cat' config 2; 13 = LineMOD all; 5 = the ClearGrasp-sized head)")
    ap.add_argument("--frame", default="480x640", help="source frame HxW (config 5: 960x1280)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--cpu-baseline-s", type=float, default=15.0)
    ap.add_argument("--breakdown", default="", help="write the per-kernel breakdown JSON here")
    ap.add_argument("--micro", type=int, default=1,
                    help="micro-batches processed concurrently inside each step (pipeline.py)")
    ap.add_argument("--flat", action="store_true", help="no plan side streams inside a micro-batch")
    ap.add_argument("--pipeline", choices=["none", "backbone", "heads", "pose"], default="heads",
                    help="two-stage pipeline (pipeline.PipelinedPipeline) split after the backbone, the heads "
                         "(default: 16.0-16.3 vs 16.3-16.5 ms/step) or before get_pose: stage A of batch k+1 runs "
                         "beside stage B of batch k; none: one batch per step end to end")
    args = ap.parse_args()

    rank, world, local = kd.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B, S, N = args.batch, args.size, args.points

    C = args.classes
    frame = tuple(int(v) for v in args.frame.split("x"))
    cfg = make_config(num_cls=C, backbone=args.backbone)
    model = KRRN(cfg=cfg)
    init_weights(model, 0)
    model = model.to(dev).eval()
    model.perm_mode = "device"
    data = make_batch(B, S, N, seed=1 + rank, objlist=list(OBJ_DICT.values())[:C] if C > 1 else None, frame=frame)
    if args.pipeline == "none" or args.micro > 1:
        step = BatchPipeline(model, B, S, N, dev, parts=args.micro, seed=rank, inner_streams=not args.flat)
    else:
        step = PipelinedPipeline(model, B, S, N, dev, seed=rank, split=args.pipeline)
    step.load(data)
    record = torch.zeros((B, kd.RECORD), dtype=torch.float32, device=dev)

    step.run()  # eager warm-up (compiles nothing; touches every buffer)
    torch.cuda.synchronize()
    if not args.no_graph:
        step.capture()

    def one_step():
        step.step()
        if world > 1:
            r = step.results()  # the batch this step completed
            kd.pack_records(r["R"], r["t"], r["pred_t"], r["inliers"], out=record)
            kd.gather_records(record)

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el

    roof, breakdown = None, None
    if rank == 0 and not args.no_profile:
        step.profile()  # warm the eager path once
        prof = step.profile()
        roof, breakdown = roofline_from_profile(prof, B)
        fids = set().union(*(getattr(pt.kp, "fusion_op_ids", set()) for pt in step.parts))
        roof["fusion"] = fusion_roofline(prof, fids, B, N)
        if args.breakdown:
            with open(args.breakdown, "w") as f:
                json.dump({"roofline": roof, "kernels": breakdown}, f, indent=1)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_s > 0:
        cpu = cpu_baseline(2, S, N, args.backbone, args.cpu_baseline_s)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "crops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded LineMOD-shaped crops, random-init weights)",
            "config": {"workload": (f"LineMOD 'cat'" if C == 1 else f"{C}-class") +
                                   f" batch={B}/GPU, {S}x{S} crops from {frame[1]}x{frame[0]} RGB-D, "
                                   f"HRNet-{args.backbone.upper()} + {N}-pt fusion + TBase, PnP-RANSAC (H=100) on GPU",
                       "batch_per_gpu": B, "crop": S, "points": N, "backbone": f"hrnet_{args.backbone}",
                       "parallelism": f"dp{world}" if world > 1 else "single", "graph": step.graph is not None,
                       "micro_batches": args.micro,
                       "pipeline": "none" if isinstance(step, BatchPipeline) else
                       f"2-stage split after the {args.pipeline} (stage A of batch k+1 beside stage B of batch k; "
                       "one batch completes per step)"},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
