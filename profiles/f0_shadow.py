"""Where does the wrong F0 of the cross-graph mismatch come from?

The round-3 finding: with the two-slot pipeline's stage graphs replayed side by side
(KRRN_STREAMS=1), F0 (the level-0 Conv_surface output) of slot 0 differed from a serial re-run in
65-98 points while its inputs were bit-identical at the end. Two mechanisms fit: the surface conv
produced the wrong values (it read something stale), or a store from elsewhere overwrote F0 after
it was produced. This script tells them apart: right after each branch's surface conv, a copy op on
the same stream writes that F0 slice into a shadow buffer (the value as produced). After a graph
half-step:
  shadow == serial, F0 != serial  -> F0 was overwritten after it was produced;
  shadow != serial                 -> the surface conv itself produced wrong values (or a store
                                      landed between it and the copy).
It also reports the wrong entries' values against zero and against the other slot's F0 (the two
slots load different batches here, so a value read across slots is recognisable). Before every
graph half-step both slots' F0 and shadows are filled with sentinels (-7 / -9): F0 is recomputed
from the same inputs each rep, so a lost store or a read of a stale copy would otherwise show the
previous rep's identical value; with the sentinel, a store that never reached memory reads -7.

usage (GPU box, the diagnostics build of the library):
  make -C pose_estimation_amd/csrc diag
  KRRN_STREAMS=1 python3 profiles/f0_shadow.py [REPS] [--history]"""
import ctypes
import os
import sys

os.environ.setdefault("KRRN_STREAMS", "1")
# krrn_gcn_debug exists only in the diagnostics build (csrc/krrn_diag.h)
os.environ.setdefault("KRRN_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "build", "diag", "libkrrn_hip_diag.so"))
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pose_estimation_amd import KRRN, _lib, make_config  # noqa: E402
from pose_estimation_amd.pipeline import PipelinedPipeline, _sub_plan  # noqa: E402
from pose_estimation_amd.runtime import Late, Op, P, ptr, _skey  # noqa: E402
from pose_estimation_amd.synthetic import init_weights, make_batch  # noqa: E402

_lib.register("krrn_gcn_debug", [P, ctypes.c_int, ctypes.c_longlong])

args = [a for a in sys.argv[1:] if not a.startswith("--")]
REPS = int(args[0]) if args else 5
dev = torch.device("cuda", 0)
print(f"KRRN_STREAMS={os.environ['KRRN_STREAMS']}", flush=True)
if "--history" in sys.argv:
    # the history under which tests/test_gpu_pipeline.py::test_pipelined_graph_benched_shape failed:
    # the file's other tests first, in order (as profiles/race_bench_shape.py)
    import test_gpu_pipeline as tgp  # noqa: E402
    for name, a in (("test_pipeline_matches_api_and_graph", (1,)), ("test_pipeline_matches_api_and_graph", (2,)),
                    ("test_pipelined_matches_plain", ("backbone",)), ("test_pipelined_matches_plain", ("heads",)),
                    ("test_pipelined_matches_plain", ("pose",)),
                    ("test_pipelined_matches_plain_after_history", ("heads",)),
                    ("test_pipelined_matches_plain_after_history", ("backbone",))):
        try:
            getattr(tgp, name)(dev, *a)
            print(f"{name}{a}: ok", flush=True)
        except AssertionError as e:
            print(f"{name}{a}: MISMATCH {str(e)[:120]}", flush=True)
    torch.cuda.synchronize()
B, S, N = 64, 120, 1000
m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
init_weights(m, 0)
m = m.to(dev).eval()
pp = PipelinedPipeline(m, B, S, N, dev, seed=0, split="heads")
for si, sl in enumerate(pp.slots):
    sl.load(make_batch(B, S, N, seed=1 + si))

# shadow copies right after each surface conv (krrn_gcn_conv_f32 with Y == NULL) of both slots
shadows = []
for si, sl in enumerate(pp.slots):
    kp = sl.parts[0].kp
    F0 = kp.fusion_bufs["F0"]
    sh = torch.zeros_like(F0)
    kp.plan.buffers.append(sh)
    shadows.append(sh)
    ops = kp.plan.ops
    i = 0
    while i < len(ops):
        op = ops[i]
        if isinstance(op, Op) and op.name == "krrn_gcn_conv_f32" and op.args[10].value is None:
            out = op.args[14].value
            co = (out - F0.data_ptr()) // 4
            cp = Op("krrn_add_relu_f32", [P(F0.data_ptr() + 4 * co), 384, 0, P(0), 0, 0, P(sh.data_ptr() + 4 * co), 384,
                                          0, B * N, 128, 0, Late(_skey(op.sid))], sid=op.sid)
            ops.insert(i + 1, cp)
            i += 1
        i += 1
# the stage views were cut before the insertion: rebuild them
for si, sl in enumerate(pp.slots):
    kp = sl.parts[0].kp
    cut = kp.heads_end
    pp.stage_a[si] = [(_sub_plan(kp.plan, 0, cut), kp.env)]
    pp.stage_b[si] = [(kp.device_perm_plan, {}), (_sub_plan(kp.plan, cut, len(kp.plan.ops)), kp.env),
                      (sl.parts[0].pose, {})]
s0 = [sl.parts[0].kp.seed.clone() for sl in pp.slots]
pp.run()
torch.cuda.synchronize()
# surface-conv input dumps (krrn_gcn_debug): per (crop, point, neighbour) the neighbour index and the
# coordinates the kernel read. capture() runs B(0), A(0), B(1), A(1) eagerly, then captures them in
# that order: launches 0-5 and again 6-11 -> slots 0-2 = slot 0's v / x / n branches, 3-5 = slot 1's
K0 = 10
GX = -(-N // 8)  # blocks per crop of the surface conv (8 points per block)
REC = B * N * K0 * 8
NBLK = B * GX
WORDS = REC + 20 * NBLK + 16384 * NBLK
if "--retouch" in sys.argv:
    # rewrite every plan-owned tensor through a device kernel (read + write back through the L2s)
    # before the captures: tells constants written by host-to-device copies from kernel-written ones
    import write_audit  # noqa: E402
    seen = set()
    for sl in pp.slots:
        ts = []
        write_audit._flatten(sl.parts[0].kp.plan.buffers, ts, set())
        for t in ts:
            if t.is_cuda and t.data_ptr() not in seen and t.numel():
                seen.add(t.data_ptr())
                t.copy_(t.clone())
    torch.cuda.synchronize()
    print(f"retouched {len(seen)} plan tensors", flush=True)
dump_g = torch.zeros(6 * WORDS, dtype=torch.int32, device=dev)
dump_s = torch.zeros(3 * WORDS, dtype=torch.int32, device=dev)
_lib.call("krrn_gcn_debug", ptr(dump_g), 6, WORDS)
pp.capture()
_lib.call("krrn_gcn_debug", P(0), 1, 1)
kp0 = pp.slots[0].parts[0].kp
P9, IDX0 = kp0.p9, kp0.fusion_bufs["idx0"]
F0s = [sl.parts[0].kp.fusion_bufs["F0"] for sl in pp.slots]
bad_reps = 0
for rep in range(REPS):
    for sl, s in zip(pp.slots, s0):
        sl.parts[0].kp.seed.copy_(s)
    pp.reset()
    for f, sh in zip(F0s, shadows):
        f.fill_(-7.0)
        sh.fill_(-9.0)
    torch.cuda.synchronize()
    pp.step()  # B(0) beside A(1)
    torch.cuda.synchronize()
    f0g, shg, f01 = F0s[0].clone(), shadows[0].clone(), F0s[1].clone()
    p9g, idxg, dg = P9.clone(), IDX0.clone(), dump_g[:3 * WORDS].clone()
    pp.slots[0].parts[0].kp.seed.copy_(s0[0])
    _lib.call("krrn_gcn_debug", ptr(dump_s), 3, WORDS)
    pp._run_b(0)  # serial re-run of slot 0's stage B from the same state
    torch.cuda.synchronize()
    _lib.call("krrn_gcn_debug", P(0), 1, 1)
    f0s = F0s[0].clone()
    print(f"   after the graph step vs the serial re-run: p9 differs at {int((p9g != P9).sum())}, idx0 at "
          f"{int((idxg != IDX0).sum())} entries", flush=True)
    for br in range(3):
        g_ = dg[br * WORDS:br * WORDS + REC].view(B, N, K0, 8)
        s_ = dump_s[br * WORDS:br * WORDS + REC].view(B, N, K0, 8)
        gb = dg[br * WORDS + REC:br * WORDS + REC + 20 * NBLK].view(NBLK, 20)
        sb = dump_s[br * WORDS + REC:br * WORDS + REC + 20 * NBLK].view(NBLK, 20)
        gt = dg[br * WORDS + REC + 20 * NBLK:(br + 1) * WORDS].view(torch.float32).view(NBLK, 256, 8, 8)
        st_ = dump_s[br * WORDS + REC + 20 * NBLK:(br + 1) * WORDS].view(torch.float32).view(NBLK, 256, 8, 8)
        da_ = (gb[:, 6:14] != sb[:, 6:14]).any(-1)
        print(f"   branch {br}: blocks whose kernel arguments differ from the serial run's: {int(da_.sum())}; "
              f"distinct argument sets in the graph {len(set(map(tuple, gb[:, 6:14].tolist())))}", flush=True)
        de_g = (gb[:, 16:20] != gb[:, 0:4]).any(-1)
        de_s = (sb[:, 16:20] != sb[:, 0:4]).any(-1)
        print(f"   branch {br}: blocks whose LDS changed during the support loop: graph {int(de_g.sum())}, serial "
              f"{int(de_s.sum())}; point-direction digest differs graph vs serial before the loop in "
              f"{int((gb[:, 2:4] != sb[:, 2:4]).any(-1).sum())} blocks", flush=True)
        dd_ = (gb[:, :2] != sb[:, :2]).any(-1)
        wrong_pts = (f0g[..., 128 * br:128 * (br + 1)] != f0s[..., 128 * br:128 * (br + 1)]).any(-1)  # [B, N]
        wb = sorted({int(b_) * GX + int(p_) // 8 for b_, p_ in wrong_pts.nonzero().tolist()})
        xg = (gb[:, 4] & 0xF).tolist()
        print(f"   branch {br}: blocks whose staged-direction digest differs from the serial run: {int(dd_.sum())} "
              f"of {B * GX} (XCDs {sorted(set(xg[i] for i in dd_.nonzero().flatten().tolist()))}); distinct graph "
              f"digests {len(set(map(tuple, gb[:, :2].tolist())))}, serial {len(set(map(tuple, sb[:, :2].tolist())))}; "
              f"blocks holding wrong F0 points {len(wb)}, their XCDs {sorted(set(xg[i] for i in wb))}, digest differs in "
              f"{sum(int(dd_[i]) for i in wb)}", flush=True)
        print(f"   branch {br}: of the blocks holding wrong points, LDS changed during the loop in "
              f"{sum(int(de_g[i]) for i in wb)}", flush=True)
        # per (thread, support): the support max and the first weight quad as held in registers
        Sn = 7
        dm = (gt[:, :, :Sn, 0:4] != st_[:, :, :Sn, 0:4]).any(-1)   # [NBLK, 256, S]
        dw = (gt[:, :, :Sn, 4:8] != st_[:, :, :Sn, 4:8]).any(-1)
        print(f"   branch {br}: (thread, support) records whose max differs {int(dm.sum())}, whose weight quad "
              f"differs {int(dw.sum())}; both {int((dm & dw).sum())}", flush=True)
        for blk, th_, s_ in dm.nonzero()[:6].tolist():
            w_prev = st_[blk, th_, s_ - 1, 4:8].tolist() if s_ > 0 else None
            print(f"     blk {blk} thr {th_} s {s_}: max g {gt[blk, th_, s_, 0:4].tolist()} s {st_[blk, th_, s_, 0:4].tolist()}"
                  f" | w g {gt[blk, th_, s_, 4:8].tolist()} s {st_[blk, th_, s_, 4:8].tolist()} (serial w at s-1 {w_prev})",
                  flush=True)
        for i in wb[:3]:
            print(f"     block {i}: graph {gb[i].tolist()} serial {sb[i].tolist()}", flush=True)
        d_nb = g_[..., 0] != s_[..., 0]
        d_pi = (g_[..., 1:4] != s_[..., 1:4]).any(-1)
        d_nj = (g_[..., 4:7] != s_[..., 4:7]).any(-1)
        print(f"   branch {br} as read by the surface conv (graph vs serial): neighbour index differs at "
              f"{int(d_nb.sum())}, point coords at {int(d_pi.sum())}, neighbour coords at {int(d_nj.sum())} of "
              f"{d_nb.numel()} (crop, point, j)", flush=True)
        bad = (d_nb | d_pi | d_nj).nonzero()[:6].tolist()
        for b_, p_, j_ in bad:
            gr, sr = g_[b_, p_, j_].tolist(), s_[b_, p_, j_].tolist()
            f = lambda w: [round(float(torch.tensor(w, dtype=torch.int32).view(torch.float32)), 7) for w in w]  # noqa: E731
            print(f"     [{b_},{p_},{j_}] graph nb {gr[0]} p {f(gr[1:4])} nb {f(gr[4:7])} | serial nb {sr[0]} "
                  f"p {f(sr[1:4])} nb {f(sr[4:7])}", flush=True)
    d_f0 = (f0g != f0s)
    d_sh = (shg != f0s)
    print(f"rep {rep}: F0(graph) != F0(serial) at {int(d_f0.sum())} entries / {int(d_f0.any(-1).sum())} points; "
          f"shadow(graph) != F0(serial) at {int(d_sh.sum())} entries; shadow != F0(graph) at "
          f"{int((shg != f0g).sum())}", flush=True)
    if d_f0.any() or d_sh.any():
        bad_reps += 1
        dd = d_f0 | d_sh
        for sl3 in range(3):
            part = dd[..., 128 * sl3:128 * (sl3 + 1)]
            pts = part.any(-1).nonzero()
            print(f"   slice {sl3}: {int(part.sum())} entries, {len(pts)} points, first (crop, point) "
                  f"{pts[:6].tolist()}", flush=True)
        idx = dd.nonzero()[:12]
        for b, n, c in idx.tolist():
            print(f"   [{b},{n},{c}] serial {float(f0s[b, n, c]):+.6e} graph {float(f0g[b, n, c]):+.6e} "
                  f"shadow {float(shg[b, n, c]):+.6e} slot1 {float(f01[b, n, c]):+.6e}", flush=True)
        wrong = f0g[d_f0]
        if wrong.numel():
            # where else do the wrong values occur in the serial F0 (another point / slice / crop)?
            flat = f0s.flatten()
            hits = 0
            for k_, (b_, n_, c_) in enumerate(d_f0.nonzero().tolist()[:40]):
                w_ = f0g[b_, n_, c_]
                pos = (flat == w_).nonzero().flatten().tolist()
                hits += bool(pos)
                if k_ < 8:
                    wh = [(q // (N * 384), (q // 384) % N, q % 384) for q in pos[:3]]
                    print(f"     wrong [{b_},{n_},{c_}] = {float(w_):+.7e} found in serial F0 at {wh}", flush=True)
            print(f"   {hits} of {min(40, wrong.numel())} wrong values occur somewhere in the serial F0", flush=True)
            print(f"   wrong F0 values: zero {int((wrong == 0).sum())} of {wrong.numel()}; equal to slot-1 F0 "
                  f"{int((f0g[d_f0] == f01[d_f0]).sum())}; sentinel (store lost) {int((wrong == -7.0).sum())}",
                  flush=True)
        wsh = shg[d_sh]
        if wsh.numel():
            print(f"   wrong shadow values: sentinel (copy lost) {int((wsh == -9.0).sum())}, F0 sentinel read "
                  f"{int((wsh == -7.0).sum())} of {wsh.numel()}", flush=True)
print(f"{bad_reps} of {REPS} half-steps mismatched", flush=True)
