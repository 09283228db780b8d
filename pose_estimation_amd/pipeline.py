"""Fixed-shape batch pipeline: KRRN forward + get_pose as one graph-capturable step.

This is the eval loop of tools/trainer.py:440-480 (forward, then get_pose per crop) for a
whole batch, with the device-side randomness the reference draws on the host (Pool_layer
randperms, the 256-point PnP subset, the RANSAC hypotheses), so a step needs no host sync and
can be captured once into a hipGraph and replayed.

Micro-batch concurrency (parts > 1): the batch is split into `parts` equal slices, each with
its own compiled plan, run side by side on their own streams inside the same step. The HRNet
low-resolution branches, the GCN levels and PnP are latency-bound (small grids, long
dependency chains) while the S=120 head convs are MFMA-bound; running two slices at once
lets one slice's latency-bound phases fill the CUs the other's big GEMMs leave idle. Every
crop of the batch is still processed exactly once per step, with the same per-crop math.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from .krrn import KRRN, KRRNPlan
from .pose import add_pose_ops
from .runtime import STREAMS, Plan, ptr


@dataclass
class _Part:
    kp: KRRNPlan
    pose: Plan
    xm: torch.Tensor
    ym: torch.Tensor
    K4: torch.Tensor
    ext: torch.Tensor
    lfb: torch.Tensor
    R: torch.Tensor
    t: torch.Tensor
    inl: torch.Tensor
    lo: int
    hi: int
    aux: Dict[str, torch.Tensor]  # the device-drawn PnP subset / RANSAC subsets / inlier mask


class BatchPipeline:
    def __init__(self, model: KRRN, B: int, S: int, N: int, device, parts: int = 1, seed: int = 0,
                 inner_streams: bool = True, pose_stream: bool = True, pose_in_plan: bool = True):
        """pose_in_plan: get_pose's launches inside the forward plan on their own stream (default),
        or as the separate `pose` plan after it (PipelinedPipeline(split='pose'))."""
        if B % parts:
            raise ValueError(f"batch {B} not divisible into {parts} parts")
        self.B, self.S, self.N, self.device = B, S, N, torch.device(device)
        b = B // parts
        self.parts: List[_Part] = []
        for p in range(parts):
            dev = self.device
            xm = torch.zeros((b, N), device=dev)
            ym = torch.zeros((b, N), device=dev)
            K4 = torch.zeros((b, 4), device=dev)
            ext = torch.zeros((b, 3), dtype=torch.float64, device=dev)
            lfb = torch.zeros((b, 3), dtype=torch.float64, device=dev)
            res = {}

            def hook(kp, res=res, xm=xm, ym=ym, K4=K4, ext=ext, lfb=lfb):
                res["pose"] = add_pose_ops(kp.plan, kp.xyz, kp.choose.view(b, N), b, N, xm, ym, K4, ext, lfb, kp.seed)

            with torch.no_grad():
                kp = KRRNPlan(model, b, S, N, True, self.device, pose_hook=hook if pose_in_plan else None,
                              pose_stream=pose_stream)
            kp.seed.fill_(1000003 * (seed + 1) + 7919 * p)
            pose = Plan(dev)  # after the forward plan: every reader of the seed has run
            if not pose_in_plan:
                res["pose"] = add_pose_ops(pose, kp.xyz, kp.choose.view(b, N), b, N, xm, ym, K4, ext, lfb, kp.seed)
            R, t, inl, aux = res["pose"]
            pose.add("krrn_rng_advance", ptr(kp.seed))
            self.parts.append(_Part(kp, pose, xm, ym, K4, ext, lfb, R, t, inl, p * b, (p + 1) * b, aux))
        self.streams = [torch.cuda.Stream(self.device) for _ in range(parts)] if parts > 1 else []
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # parts > 1 runs each part's plan serially on its part stream: capturing nested plan side
        # streams under per-part streams segfaults in hipStreamEndCapture (measured on ROCm 7.2,
        # also when every side stream first joins the capture through the origin stream)
        self.inner_streams = inner_streams and parts == 1

    # -- inputs / outputs ------------------------------------------------------------------
    def load(self, data: Dict[str, torch.Tensor]):
        """Copy one batch (PoseDataset item keys, batchdataset.py:730-771) into the static
        buffers. Host tensors are copied asynchronously on the current stream."""
        N = self.N
        for pt in self.parts:
            sl = slice(pt.lo, pt.hi)
            b = pt.hi - pt.lo
            pt.kp.load_inputs(data["img_croped"][sl].to(self.device), data["cloud"][sl].to(self.device),
                              data["choose"][sl].to(self.device), data["cls_id"][sl].to(self.device))
            pt.xm.copy_(data["x_map_choosed"][sl].reshape(b, N), non_blocking=True)
            pt.ym.copy_(data["y_map_choosed"][sl].reshape(b, N), non_blocking=True)
            pt.K4.copy_(data["intrinsic"][sl].reshape(b, 4), non_blocking=True)
            pt.ext.copy_(data["extent"][sl].reshape(b, 3), non_blocking=True)
            pt.lfb.copy_(data["lfborder"][sl].reshape(b, 3), non_blocking=True)

    def results(self) -> Dict[str, torch.Tensor]:
        """R [B,3,3], t [B,3] (PnP), pred_t [B,3] (TBase), inliers [B] of the last step."""
        cat = lambda xs: xs[0] if len(xs) == 1 else torch.cat(xs)  # noqa: E731
        return {"R": cat([p.R for p in self.parts]), "t": cat([p.t for p in self.parts]),
                "pred_t": cat([p.kp.pred_t for p in self.parts]), "inliers": cat([p.inl for p in self.parts])}

    def plans(self):
        """(plan, env) pairs of every launch list, in step order (per part)."""
        out = []
        for pt in self.parts:
            out += [(pt.kp.device_perm_plan, {}), (pt.kp.plan, pt.kp.env), (pt.pose, {})]
        return out

    # -- execution -------------------------------------------------------------------------
    def _run_part(self, pt: _Part, serial: bool):
        pt.kp.device_perm_plan.run({}, serial=serial)
        pt.kp.plan.run(pt.kp.env, serial=serial)
        pt.pose.run({}, serial=serial)

    def run(self, concurrent: bool = False):
        """Enqueue one step on the current stream. Eagerly everything runs serially on it; with
        `concurrent` (used under hipGraph capture only, see runtime.Plan) the plans' side streams
        and the micro-batches' streams fork and join back."""
        serial = not concurrent
        if not self.streams or serial or not STREAMS:
            # one part after the other on the caller's stream (under capture each part's plan keeps
            # its graph branches; parts side by side on their streams only with KRRN_STREAMS=1)
            for pt in self.parts:
                self._run_part(pt, serial)
            return
        main = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(main)
        for pt, s in zip(self.parts, self.streams):
            with torch.cuda.stream(s):
                self._run_part(pt, not self.inner_streams)
        for s in self.streams:
            main.wait_stream(s)

    def capture(self):
        """Warm up once, then capture one step into a hipGraph."""
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self.run()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.run(concurrent=True)
        torch.cuda.synchronize(self.device)

    def step(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self.run()

    def profile(self):
        """Per-op device time of one serial step (HIP events around every launch)."""
        out = []
        for p, env in self.plans():
            out.extend(p.run_timed(dict(env)))
        return out


# ------------------------------------------------------------------------------------------
# Two-stage software pipeline across batches
# ------------------------------------------------------------------------------------------
def _sub_plan(plan: Plan, lo: int, hi: int) -> Plan:
    """A view of plan.ops[lo:hi] sharing the plan's side streams."""
    sub = Plan(plan.device)
    sub.ops, sub.nstreams, sub._side = plan.ops[lo:hi], plan.nstreams, plan._side
    return sub


class PipelinedPipeline:
    """BatchPipeline's step as a two-stage software pipeline over two batch slots.

    Stage A = the HRNet backbone (KRRNPlan.ops[:split]: ~430 small, latency-bound convs that
    leave most CUs idle), stage B = heads + fusion + TBase + PnP (KRRNPlan.ops[split:] plus the
    device draws and the pose plan). Half-step h runs B of slot h on the caller's stream while A
    of slot 1-h runs on a side stream; each stage of each slot is its own hipGraph (one capture
    per stage: capturing both into one graph would need side streams forking side streams, which
    segfaults in hipStreamEndCapture on ROCm 7.2), and a half-step replays two of them on two
    streams. In steady state every half-step completes one whole batch (`results()`); a crop's
    math is unchanged (same kernels, per-slot buffers), only its latency is two half-steps.
    """

    def __init__(self, model: KRRN, B: int, S: int, N: int, device, seed: int = 0, split: str = "backbone"):
        """split: 'backbone' (A = HRNet), 'heads' (A = HRNet + heads + class select, B = the
        latency-bound fusion / TBase / PnP tail) or 'pose' (A = the whole forward, B = get_pose:
        the PnP-RANSAC of batch k, long-lived and LDS-heavy, runs beside the latency-bound
        backbone of batch k+1 instead of the fusion / TBase tail of batch k)."""
        self.B, self.S, self.N, self.device = B, S, N, torch.device(device)
        self.slots = [BatchPipeline(model, B, S, N, device, parts=1, seed=2 * seed + i, pose_in_plan=split != "pose")
                      for i in range(2)]
        self.stage_a: List[List[Tuple[Plan, dict]]] = []
        self.stage_b: List[List[Tuple[Plan, dict]]] = []
        for sl in self.slots:
            pt = sl.parts[0]
            kp = pt.kp
            if split == "pose":
                self.stage_a.append([(kp.device_perm_plan, {}), (kp.plan, kp.env)])
                self.stage_b.append([(pt.pose, {})])
                continue
            cut = {"backbone": kp.split, "heads": kp.heads_end}[split]
            self.stage_a.append([(_sub_plan(kp.plan, 0, cut), kp.env)])
            self.stage_b.append([(kp.device_perm_plan, {}), (_sub_plan(kp.plan, cut, len(kp.plan.ops)), kp.env),
                                 (pt.pose, {})])
        self.side = torch.cuda.Stream(self.device)
        self.graphs_a: List[Optional[torch.cuda.CUDAGraph]] = [None, None]
        self.graphs_b: List[Optional[torch.cuda.CUDAGraph]] = [None, None]
        self.h = 0
        self.primed = False

    def load(self, data):
        for s in self.slots:
            s.load(data)

    def _run_a(self, slot: int, concurrent: bool = False):
        for p, env in self.stage_a[slot]:
            p.run(dict(env), serial=not concurrent)

    def _run_b(self, slot: int, concurrent: bool = False):
        for p, env in self.stage_b[slot]:
            p.run(dict(env), serial=not concurrent)

    def _prime(self):
        """Stage A of both slots once, so the first half-step's stage B has backbone features."""
        for i in range(2):
            self._run_a(i)
        self.primed = True

    def _half(self, run_a, run_b):
        b, a = self.h, self.h ^ 1
        if not STREAMS:  # the two stages one after the other on the caller's stream (runtime.Plan)
            run_b(b)
            run_a(a)
            self.h ^= 1
            return
        main = torch.cuda.current_stream(self.device)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            run_a(a)
        run_b(b)
        main.wait_stream(self.side)
        self.h ^= 1

    def reset(self):
        """Re-run stage A of both slots (eager) from the current RNG state; the next half-step
        completes slot 0."""
        self._prime()
        self.h = 0

    def run(self):
        """One eager half-step: stage B of slot h, THEN stage A of the other slot, both on the
        caller's stream (no concurrency between the two slots' launch lists).

        Run side by side eagerly, the two slots' plans enqueue onto ~14 HIP streams, more than the
        GPU_MAX_HW_QUEUES = 4 hardware queues the runtime multiplexes them onto; under that sharing
        a stage-B kernel intermittently consumed an input its own stream's previous kernel had not
        finished publishing (profiles/race_bisect.py, DESIGN.md §5: 4/5 mismatching half-steps with
        4 hardware queues, 0/5 with 16, 0/5 with either stage on one stream, 0/5 sequential, 0/5 as
        captured hipGraphs). The concurrent form is the graph replay (`step` after `capture`);
        eagerly each stage also runs serially (runtime.Plan.run)."""
        if not self.primed:
            self._prime()
        b, a = self.h, self.h ^ 1
        self._run_b(b)
        self._run_a(a)
        self.h ^= 1

    def capture(self):
        """Warm up every stage once on a side stream, then capture one hipGraph per stage and slot."""
        if not self.primed:
            self._prime()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for i in range(2):
                self._run_b(i)
                self._run_a(i)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for i in range(2):
            for gs, fn in ((self.graphs_b, self._run_b), (self.graphs_a, self._run_a)):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    fn(i, concurrent=True)
                gs[i] = g
        torch.cuda.synchronize(self.device)
        # the captures above do not execute: slot state is as after the warm-up (A of both slots
        # last), so the next half-step's stage B (slot 0) reads valid features
        self.h = 0

    def step(self):
        if self.graphs_a[0] is None:
            self.run()
            return
        self._half(lambda i: self.graphs_a[i].replay(), lambda i: self.graphs_b[i].replay())

    def results(self):
        """The batch completed by the most recent half-step."""
        return self.slots[self.h ^ 1].results()

    def plans(self):
        return self.slots[0].plans()

    def profile(self):
        return self.slots[0].profile()

    @property
    def graph(self):
        return self.graphs_a[0]

    @property
    def parts(self):
        return self.slots[0].parts
