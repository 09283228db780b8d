"""KRRN inference benchmark on MI355X (BASELINE.json metric: crops/s).

A step = one pass of the hot path over one batch of synthetic LineMOD crops resident in HBM:
HRNet-W18 + heads + class select/normalise + choose gather + FusionNetLite + TBase (pred_t)
+ batched PnP-RANSAC (R), including the device-side randomness (pool permutations, the 256-
point PnP subset, RANSAC hypotheses). The step is one hipGraph replay of the whole path (the plan's
independent branches as graph branches, runtime.Plan); the two-slot pipeline (--pipeline
heads|backbone|pose) and concurrent micro-batches replay side by side on two streams (KRRN_STREAMS=1,
the default since the round-4 root cause) and measured no faster. With --gpus N
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
from pose_estimation_amd.runtime import PLAN_STREAMS, STREAMS  # noqa: E402
from pose_estimation_amd.synthetic import OBJ_DICT, init_weights, make_batch  # noqa: E402

METRIC = "crops/sec at 640×480 RGB-D, 1000 sampled pts; ADD(-S) AUC vs reference"
PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32-input MFMA (= f32 vector peak)
PEAK_BF16_MFMA_TFLOPS = 2516.6  # MI355X_MICROARCH.md: dense bf16 MFMA, 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz
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
        g = groups.setdefault(k, {"ms": 0.0, "flops": 0.0, "mfma": 0.0, "bf16": 0.0, "n": 0})
        g["ms"] += ms
        g["flops"] += op.meta.get("flops", 0.0)
        g["mfma"] += op.meta.get("mfma_flops", op.meta.get("flops", 0.0))
        g["bf16"] += op.meta.get("mfma_bf16_flops", 0.0)
        g["n"] += 1
    total_ms = sum(g["ms"] for g in groups.values())
    dom = max(groups, key=lambda k: groups[k]["ms"])
    g = groups[dom]
    avg_ms = g["ms"] / g["n"]
    achieved = (g["flops"] / g["n"]) / (avg_ms * 1e-3) / 1e12 if g["flops"] > 0 else None
    conv_ms = sum(v["ms"] for k, v in groups.items() if k.startswith("conv_gemm"))
    conv_fl = sum(v["flops"] for k, v in groups.items() if k.startswith("conv_gemm"))
    allc = [v for k, v in groups.items() if k.startswith(("conv_gemm", "conv_group", "convt", "wino", "hipblaslt"))]
    allc_ms, allc_fl, allc_mf = (sum(v[f] for v in allc) for f in ("ms", "flops", "mfma"))
    breakdown = {k: {"ms": round(v["ms"], 4), "launches": v["n"],
                     **({"TFLOP/s": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2)} if v["flops"] else {})}
                 for k, v in sorted(groups.items(), key=lambda kv: -kv[1]["ms"])}
    traffic, tsrc = _pmc_traffic(dom)
    # achieved = ALGORITHMIC FLOPs per launch (SURVEY §8d's direct-conv formula 2 Cin Cout 9 M) /
    # the average launch time, against the dense peak of the matrix pipe the kernel runs on (bf16 for
    # the split kernels): the roofline fraction of the work. pipe_achieved / pipe_frac = what the
    # matrix pipe actually issues (Winograd F(2x2,3x3): 16/36 of the direct multiplies; split-bf16:
    # 6 bf16 term products per f32 product) -- pipe occupancy, not work
    bf16 = g["bf16"] > 0
    pipe_fl, peak = (g["bf16"], PEAK_BF16_MFMA_TFLOPS) if bf16 else (g["mfma"], PEAK_F32_MFMA_TFLOPS)
    mp = (pipe_fl / g["n"]) / (avg_ms * 1e-3) / 1e12 if pipe_fl > 0 else None
    roof = {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 2) if achieved else None,
            "peak": peak, "unit": "TFLOP/s", "pipe": "bf16 (f32-accurate 3-term split)" if bf16 else "f32",
            "frac": round(achieved / peak, 4) if achieved else None,
            "pipe_achieved": round(mp, 2) if mp else None, "pipe_frac": round(mp / peak, 4) if mp else None,
            "traffic": traffic,
            "traffic_unit": "HBM bytes per launch", "traffic_source": tsrc,
            "launches": g["n"], "avg_launch_us": round(avg_ms * 1e3, 2),
            "mfma_flops_per_launch": round(pipe_fl / g["n"]),
            "effective_tflops": round(achieved, 2) if achieved else None,
            "effective_flops_per_launch": round(g["flops"] / g["n"]),
            "all_conv_gemm": {"ms_per_step": round(conv_ms, 3),
                              "TFLOP/s": round(conv_fl / (conv_ms * 1e-3) / 1e12, 2) if conv_ms else None,
                              "GFLOP_per_crop": round(conv_fl / B / 1e9, 3)},
            "all_conv": {"ms_per_step": round(allc_ms, 3), "GFLOP_per_crop": round(allc_fl / B / 1e9, 3),
                         "effective_TFLOP/s": round(allc_fl / (allc_ms * 1e-3) / 1e12, 2) if allc_ms else None,
                         "mfma_pipe_TFLOP/s": round(allc_mf / (allc_ms * 1e-3) / 1e12, 2) if allc_ms else None,
                         "mfma_pipe_frac": round(allc_mf / (allc_ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4)
                         if allc_ms else None,
                         "note": "every conv / GEMM of the step incl. Winograd; effective = direct-conv FLOPs "
                                 "(SURVEY §8d), pipe = FLOPs the MFMA pipe issues in f32-MFMA time (bf16 "
                                 "FLOPs / 16)"},
            "events_ms_per_step": round(total_ms, 3)}
    return roof, breakdown


def conv_subset(prof, ids):
    """MFMA rate of the conv / GEMM launches whose op id is in `ids` (e.g. the HRNet body)."""
    ops = [(op, ms) for op, ms in prof if id(op) in ids and op.meta.get("flops")]
    if not ops:
        return None
    ms = sum(t for _, t in ops)
    fl = sum(op.meta["flops"] for op, _ in ops)
    mf = sum(op.meta.get("mfma_flops", op.meta["flops"]) for op, _ in ops)
    return {"ms_per_step": round(ms, 3), "launches": len(ops), "effective_TFLOP/s": round(fl / (ms * 1e-3) / 1e12, 2),
            "mfma_pipe_TFLOP/s": round(mf / (ms * 1e-3) / 1e12, 2),
            "mfma_pipe_frac": round(mf / (ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4)}


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


def _cpu_model_name() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs this process may use: the cgroup v2 quota (cpu.max) when set, else the affinity set.
    The GPU box reports os.cpu_count() = 256 host CPUs under a 16-CPU quota: 256 torch threads
    would oversubscribe the quota 16x, so the CPU leg uses the quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_config(B: int, S: int, N: int, backbone: str, warmup: int, reps: int, seed: int):
    """crops/s of the CPU oracle (PyTorch-CPU restatement + C EPnP-RANSAC, H = 100, 1 px) on one
    config: `warmup` untimed batches, then the median over `reps` timed batches."""
    import statistics
    from oracle.krrn_oracle import KRRNOracle, get_pose
    from pose_estimation_amd.fusion import level_sizes
    m = KRRN(cfg=make_config(num_cls=1, backbone=backbone))
    sd = init_weights(m, 0)
    o = KRRNOracle(num_cls=1, backbone=backbone)
    o.load_state_dict(sd)
    o.eval()
    d = make_batch(B, S, N, seed=99)
    N1, N2, _, _ = level_sizes(N, 10)

    def one():
        perms = [torch.randperm(N)[:N1] for _ in range(4)] + [torch.randperm(N1)[:N2]]
        pred = o(d["img_croped"], d["cloud"], d["choose"], d["cls_id"], perms=perms)
        sel = torch.stack([torch.randperm(N)[:256] for _ in range(B)])
        subs = torch.stack([torch.stack([torch.randperm(256)[:5] for _ in range(100)]) for _ in range(B)])
        get_pose(pred, d, sel, subs.int())

    times = []
    for i in range(warmup + reps):
        t0 = time.perf_counter()
        one()
        el = time.perf_counter() - t0
        print(f"[cpu leg] B={B} {backbone} iter {i}: {el:.2f} s", file=sys.stderr, flush=True)
        if i >= warmup:
            times.append(el)
    if not times:
        return {"value": None, "batch": B, "backbone": f"hrnet_{backbone}", "warmup": warmup, "reps": 0}
    med = statistics.median(times)
    return {"value": round(B / med, 4), "batch": B, "backbone": f"hrnet_{backbone}", "warmup": warmup, "reps": reps,
            "median_s_per_batch": round(med, 4)}


def cpu_baseline(S: int, N: int, threads: int, reps2: int, warmup2: int):
    """the CPU oracle on the GPU box's host cores, config 1 (B = 1, the reference's
    HRNet config.yaml widths) and config 2 (B = 64, HRNet-W18), S = 120, N = 1000, crops/s as the
    median of timed batches after warm-ups (config 1: 3 + 10; config 2: `warmup2` + `reps2`, the
    protocol's 3 + 10 by default, ~3 minutes on the GPU box's 16-CPU quota)."""
    torch.set_num_threads(threads)
    c1 = _cpu_config(1, S, N, "lm", 3, 10, 0)
    c2 = _cpu_config(64, S, N, "w18", warmup2, reps2, 0)
    return {"value": c2["value"], "unit": "crops/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model_name(), "os_cpu_count": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "cpu_quota": cpu_quota(),
            "config1": c1, "config2": c2,
            "sample": f"config 2 (value): B=64 'cat' S={S} N={N} HRNet-W18, median of {reps2} batches after {warmup2} "
                      f"warm-up; config 1: B=1 HRNet config.yaml widths, median of 10 after 3; oracle/krrn_oracle.py "
                      f"f32 + oracle/pnp_ref.c EPnP-RANSAC H=100, {threads} torch threads"}


def cpu_leg_accuracy(dev, B: int = 64, N: int = 1000, S: int = 120, seed: int = 17):
    """ADD(-S) AUC of the GPU pose step vs the CPU oracle's on known-pose scenes (the checker leg:
    the oracle is only imported here and in cpu_baseline). Scenes: synthetic.make_pnp_scene, the
    chosen pixels carry the exact normalised model coordinates of a known pose, 0.4 px noise,
    30 % outliers at U[-20, 20] px. Both sides run the same 256-point subset and the same 100
    RANSAC subsets (the GPU's device draws); both poses are scored with Metric against the GT
    (half the crops as a symmetric class: ADD-S, half ADD), AUC over max_dis = 0.1 m."""
    import numpy as np
    from oracle import pnp as opnp
    from pose_estimation_amd import pose
    from pose_estimation_amd.metric import Metric, add_metric
    from pose_estimation_amd.synthetic import make_pnp_scene
    xyz, data, Rgt, tgt = make_pnp_scene(B, N, S, seed, outlier_frac=0.3, noise_px=0.4)
    R, t, info = pose.get_pose({"xyz": xyz.to(dev)}, data, return_info=True)
    torch.cuda.synchronize()
    sel = info["sel"].cpu().long()
    subs = info["subsets"].cpu().numpy()
    Ro, to = [], []
    K4 = data["intrinsic"][0].numpy()
    for b in range(B):
        s = sel[b]
        pix = data["choose"][b, 0, s]
        obj = (xyz[b].reshape(3, -1)[:, pix].double().t() * data["extent"][b] + data["lfborder"][b]).float().numpy()
        img = np.stack([data["x_map_choosed"][b, s, 0].numpy(), data["y_map_choosed"][b, s, 0].numpy()], 1)
        r_, t_, _, _, _ = opnp.pnp_ransac(obj, img, K4, subs[b], 1.0)
        Ro.append(r_)
        to.append(t_)
    Ro = torch.from_numpy(np.stack(Ro)).float()
    to = torch.from_numpy(np.stack(to)).float()
    ext, lfb = data["extent"][0].numpy(), data["lfborder"][0].numpy()
    mp = torch.from_numpy((np.random.default_rng(5).random((B, 2600, 3)) * ext + lfb).astype(np.float32))
    target = torch.einsum("bpk,bjk->bpj", mp.double(), torch.from_numpy(Rgt)) + torch.from_numpy(tgt)[:, None]
    target = target.float()
    cls = (torch.arange(B) % 2).view(B, 1)
    metric = Metric([1])
    add_g = add_metric(R, t, mp.to(dev), target.to(dev), cls.to(dev), metric.sys).cpu().numpy()
    add_o = add_metric(Ro.to(dev), to.to(dev), mp.to(dev), target.to(dev), cls.to(dev), metric.sys).cpu().numpy()
    auc_g, auc_o = metric.cal_auc(list(add_g)), metric.cal_auc(list(add_o))
    dia = float(np.linalg.norm(ext))
    return {"auc_gpu": round(auc_g, 4), "auc_oracle": round(auc_o, 4),
            "delta_pct": round(abs(auc_g - auc_o) / max(auc_o, 1e-9) * 100.0, 4),
            "add_pass_gpu": float((add_g < 0.1 * dia).mean()), "add_pass_oracle": float((add_o < 0.1 * dia).mean()),
            "max_crop_add_delta_m": float(np.abs(add_g - add_o).max()),
            "sample": f"{B} known-pose scenes, {N} pts, 256-pt PnP subset, H=100, 0.4 px noise, 30 % outliers, "
                      "ADD-S for half the crops; AUC max_dis 0.1 m (metric.py:38-65)"}


def config3_sizes(total: int, seed: int = 0):
    """BASELINE config 3's crop sizes: `total` crops with S drawn from the LineMOD test-crop
    histogram (13,425 yolov3 detections snapped by get_square_bbox, batchdataset.py:890-923)."""
    import numpy as np
    from pose_estimation_amd.dataset import LM_CROP_HIST
    hs = np.array(list(LM_CROP_HIST.keys()))
    hp = np.array(list(LM_CROP_HIST.values()), dtype=np.float64)
    return [int(v) for v in np.random.default_rng(seed).choice(hs, size=total, p=hp / hp.sum())]


def _config3_cap(buckets: dict, world: int) -> int:
    """Rows of a rank's per-step record block: the most crops any rank holds per bucket, summed (the
    same on every rank, as all_gather_into_tensor needs; shorter ranks leave zero rows)."""
    return max(1, sum(max(kd.shard_range(n, world, r)[1] - kd.shard_range(n, world, r)[0] for r in range(world))
                      for n in buckets.values()))


def bench_config3(args, rank: int, world: int, local: int):
    """BASELINE config 3: all 13 LineMOD objects, one global batch of args.global_batch crops per step
    with crop sizes from the LineMOD histogram. Like trainer.py:521-551 (process_patch_datas) and the
    eval batcher (dataset.BucketBatcher), crops are bucketed by S; every bucket is split contiguously
    across the ranks (distributed.bucket_shard), each rank runs one captured BatchPipeline per bucket
    it holds (forward + PnP on the GPU), and the per-crop pose records of the step are all-gathered
    over RCCL. value = global crops / max-over-ranks step time (strong scaling)."""
    from pose_estimation_amd.config import LM_OBJLIST
    N = args.points
    sizes = config3_sizes(args.global_batch)
    shard = kd.bucket_shard(sizes, world, rank)
    buckets_all = {S: sizes.count(S) for S in sorted(set(sizes))}
    if args.dry_run:
        dev = torch.device("cpu")
        pipes = []
        record = torch.zeros((_config3_cap(buckets_all, world), kd.RECORD), dtype=torch.float32)
        one_step = lambda: _dry_step(record.shape[0], world, record)  # noqa: E731
        sync = lambda: None  # noqa: E731
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        model = KRRN(cfg=make_config(num_cls=13, backbone=args.backbone))
        init_weights(model, 0)
        model = model.to(dev).eval()
        pipes = []
        for S, idx in shard.items():
            pl = BatchPipeline(model, len(idx), S, N, dev, parts=1, seed=rank * 97 + S)
            pl.load(make_batch(len(idx), S, N, seed=1000 * rank + S, objlist=LM_OBJLIST))
            pl.run()
            torch.cuda.synchronize()
            pl.capture()
            pipes.append(pl)
        record = torch.zeros((_config3_cap(buckets_all, world), kd.RECORD), dtype=torch.float32, device=dev)
        # the buckets' graphs side by side on a few streams (most buckets hold 1-87 crops, each alone
        # far too small to fill the chip): longest-processing-time assignment by crops x S^2
        nst = max(1, min(args.c3_streams if STREAMS else 1, len(pipes)))
        streams = [torch.cuda.Stream(dev) for _ in range(nst)] if nst > 1 else []
        load = [0.0] * nst
        assign = [0] * len(pipes)
        for i in sorted(range(len(pipes)), key=lambda i: -pipes[i].B * pipes[i].S ** 2):
            j = min(range(nst), key=lambda j: load[j])
            assign[i] = j
            load[j] += pipes[i].B * pipes[i].S ** 2

        def run_buckets():
            if not streams:
                for pl in pipes:
                    pl.step()
                return
            main = torch.cuda.current_stream(dev)
            for s_ in streams:
                s_.wait_stream(main)
            for pl, j in zip(pipes, assign):
                with torch.cuda.stream(streams[j]):
                    pl.step()
            for s_ in streams:
                main.wait_stream(s_)

        def one_step():
            run_buckets()
            if world > 1:
                o = 0
                for pl in pipes:
                    r = pl.results()
                    b = r["R"].shape[0]
                    kd.pack_records(r["R"], r["t"], r["pred_t"], r["inliers"], out=record[o:o + b])
                    o += b
                kd.gather_records(record)
        sync = torch.cuda.synchronize
    for _ in range(args.warmup):
        one_step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev if not args.dry_run else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms = el / args.steps * 1e3
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(args.global_batch * args.steps / el, 2), "unit": "crops/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "dry run (no GPU)" if args.dry_run else
                    "synthetic (seeded LineMOD-shaped crops of the 13 objects, random-init weights)",
            "config": {"workload": f"BASELINE config 3: LineMOD all 13 objects, global batch {args.global_batch} "
                                   f"crops (S from the LineMOD test-crop histogram, bucketed by S, every bucket "
                                   f"split over {world} rank(s)), HRNet-{args.backbone.upper()} + {N}-pt fusion + "
                                   f"TBase, PnP-RANSAC (H=100) on GPU",
                       "global_batch": args.global_batch, "points": N, "buckets": buckets_all,
                       "rank0_buckets": {S: len(v) for S, v in shard.items()},
                       "backbone": f"hrnet_{args.backbone}", "classes": 13,
                       "parallelism": f"dp{world}" if world > 1 else "single", "graph": not args.dry_run},
            "roofline": None, "cpu_baseline": None,
        }
        if args.dry_run:
            line["dry_run"] = True
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N rank processes (this script, RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, one GPU each) and wait. The parent never touches the GPU, and the
    ranks are fresh child processes (no re-exec)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def _dry_step(B: int, world: int, record: torch.Tensor):
    """--dry-run stand-in for one step (no GPU): a fixed host delay for the batch, then the same
    per-crop record all-gather the real step does (gloo)."""
    time.sleep(0.002)
    R = torch.eye(3).repeat(B, 1, 1)
    t = torch.zeros(B, 3)
    kd.pack_records(R, t, t, torch.zeros(B), out=record)
    if world > 1:
        kd.gather_records(record)


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
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU leg (baseline + accuracy)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="torch threads of the CPU leg (0 = the CPUs this process may use: cgroup quota / affinity)")
    ap.add_argument("--cpu-reps", type=int, default=10, help="timed B=64 CPU batches (BASELINE.md §2 protocol: 10)")
    ap.add_argument("--cpu-warmup", type=int, default=3, help="untimed B=64 CPU batches (protocol: 3)")
    ap.add_argument("--breakdown", default="", help="write the per-kernel breakdown JSON here")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo ranks, a host-delay step and the record all-gather (launcher rehearsal)")
    ap.add_argument("--micro", type=int, default=1,
                    help="micro-batches processed concurrently inside each step (pipeline.py)")
    ap.add_argument("--flat", action="store_true", help="no plan side streams inside a micro-batch")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3],
                    help="BASELINE config: 2 = LineMOD 'cat', B crops per GPU (default; weak scaling); 3 = all 13 "
                         "LineMOD objects, ONE global batch of --global-batch crops whose sizes S are drawn from the "
                         "LineMOD test-crop histogram, bucketed by S and every bucket split across the ranks "
                         "(distributed.bucket_shard; strong scaling: the 256 crops are shared by the N GPUs)")
    ap.add_argument("--global-batch", type=int, default=256, help="config 3: crops per step over all ranks")
    ap.add_argument("--c3-streams", type=int, default=3,
                    help="config 3: streams the per-bucket graphs replay on side by side (1 = one after another)")
    ap.add_argument("--pipeline", choices=["none", "backbone", "heads", "pose"], default="none",
                    help="none (default): one batch per step end to end as one hipGraph; backbone / heads / pose: "
                         "the two-stage pipeline (pipeline.PipelinedPipeline) split there, its stages side by side on two "
                         "streams (KRRN_STREAMS=1; measured no faster than one graph)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")

    rank, world, local = kd.init_from_env("gloo" if args.dry_run else "nccl")
    if args.config == 3:
        return bench_config3(args, rank, world, local)
    B, S, N = args.batch, args.size, args.points
    C = args.classes
    frame = tuple(int(v) for v in args.frame.split("x"))
    step = None
    if args.dry_run:
        dev = torch.device("cpu")
        record = torch.zeros((B, kd.RECORD), dtype=torch.float32)
        one_step = lambda: _dry_step(B, world, record)  # noqa: E731
        sync = lambda: None  # noqa: E731
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
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
        sync = torch.cuda.synchronize

    for _ in range(args.warmup):
        one_step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    sync()
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
    extra = {}
    if rank == 0 and step is not None and not args.no_profile:
        step.profile()  # warm the eager path once
        prof = step.profile()
        roof, breakdown = roofline_from_profile(prof, B)
        parts = step.parts
        fids = set().union(*(getattr(pt.kp, "fusion_op_ids", set()) for pt in parts))
        roof["fusion"] = fusion_roofline(prof, fids, B, N)
        bids = set().union(*({id(op) for op in pt.kp.plan.ops[:pt.kp.split]} for pt in parts))
        roof["hrnet_body"] = conv_subset(prof, bids)
        extra = {"fusion_hbm_frac": (roof["fusion"] or {}).get("frac"),
                 "conv_mfma_frac": roof["all_conv"]["mfma_pipe_frac"],
                 "hrnet_conv_mfma_frac": (roof["hrnet_body"] or {}).get("mfma_pipe_frac")}
        if args.breakdown:
            with open(args.breakdown, "w") as f:
                json.dump({"roofline": roof, "kernels": breakdown}, f, indent=1)
    cpu, acc = None, None
    if rank == 0 and world == 1 and step is not None and not args.no_cpu:
        acc = cpu_leg_accuracy(dev)
        threads = args.cpu_threads or cpu_quota()
        cpu = cpu_baseline(S, N, threads, args.cpu_reps, args.cpu_warmup)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "crops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "dry run (no GPU)" if args.dry_run else
                    "synthetic (seeded LineMOD-shaped crops, random-init weights)",
            "config": {"workload": (f"LineMOD 'cat'" if C == 1 else f"{C}-class") +
                                   f" batch={B}/GPU, {S}x{S} crops from {frame[1]}x{frame[0]} RGB-D, "
                                   f"HRNet-{args.backbone.upper()} + {N}-pt fusion + TBase, PnP-RANSAC (H=100) on GPU",
                       "batch_per_gpu": B, "global_batch": B * world, "crop": S, "points": N,
                       "backbone": f"hrnet_{args.backbone}",
                       "parallelism": f"dp{world}" if world > 1 else "single",
                       "graph": step is not None and step.graph is not None,
                       "micro_batches": args.micro,
                       "pipeline": "none" if isinstance(step, BatchPipeline) or step is None else
                       f"2-stage split after the {args.pipeline} (stage A of batch k+1 "
                       f"{'beside' if STREAMS else 'after'} stage B of batch k; one batch completes per step)",
                       "graph_branches": PLAN_STREAMS},
            **extra,
            "roofline": roof, "cpu_baseline": cpu, "accuracy": acc,
        }
        if args.dry_run:
            line["dry_run"] = True
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
