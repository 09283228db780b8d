"""Exact per-op device time of one bench step: the whole step (perm draw, KRRN plan, pose plan)
is captured serially (every launch on one stream) into a hipGraph and replayed under
`rocprofv3 --kernel-trace`, so kernels neither overlap nor wait on host launch gaps. The
kernels of the last replay are then matched, in order, to the plan's ops (a split-K conv is
two kernels) and grouped by op tag / shape.

usage (GPU box):
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sgp -o run -- \
      python3 profiles/serial_graph_profile.py run
  python3 profiles/serial_graph_profile.py analyse gpurun_out/sgp/run_kernel_trace.csv [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REPLAYS = 3
TWO_KERNEL_OPS = {"krrn_pnp_ransac_f32"}  # hypothesis kernel + refine kernel


def run(B=64, S=120, N=1000, oplist="gpurun_out/sgp_ops.json"):
    import torch
    from pose_estimation_amd import KRRN, make_config
    from pose_estimation_amd.pipeline import BatchPipeline
    from pose_estimation_amd.synthetic import init_weights, make_batch
    dev = torch.device("cuda:0")
    m = KRRN(cfg=make_config(num_cls=1, backbone="w18"))
    init_weights(m, 0)
    m = m.to(dev).eval()
    st = BatchPipeline(m, B, S, N, dev, parts=1)
    st.load(make_batch(B, S, N, seed=1))
    plans = st.plans()
    for p, env in plans:
        p.run(env, serial=True)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for p, env in plans:
                p.run(env, serial=True)
    torch.cuda.synchronize()
    for _ in range(REPLAYS):
        g.replay()
    torch.cuda.synchronize()
    ops = []
    for p, _ in plans:
        for op in p.kernels():
            md = op.meta
            ops.append({"name": op.name, "kernel": md.get("kernel", op.name), "tag": md.get("tag", ""),
                        "M": md.get("M"), "N": md.get("N"), "K": md.get("K"), "flops": md.get("flops", 0.0),
                        "nk": 2 if md.get("splits", 1) > 1 or op.name in TWO_KERNEL_OPS else 1})
    os.makedirs(os.path.dirname(oplist), exist_ok=True)
    json.dump(ops, open(oplist, "w"))
    print("ops", len(ops), "kernels per replay", sum(o["nk"] for o in ops))


def analyse(trace, out=None, oplist="gpurun_out/sgp_ops.json"):
    ops = json.load(open(oplist))
    per = sum(o["nk"] for o in ops)
    rows = [r for r in csv.DictReader(open(trace)) if "anonymous namespace" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = rows[-per:]
    i = 0
    groups = defaultdict(lambda: {"us": 0.0, "n": 0, "flops": 0.0})
    tot = 0.0
    for o in ops:
        us = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last[i:i + o["nk"]])
        i += o["nk"]
        key = f'{o["kernel"]} {o["tag"]} M={o["M"]} N={o["N"]} K={o["K"]}' if o["M"] else o["kernel"]
        g = groups[key]
        g["us"] += us
        g["n"] += 1
        g["flops"] += o["flops"]
        tot += us
    span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
    res = {"busy_ms": tot / 1e3, "span_ms": span / 1e3, "groups": {}}
    print(f"serial step: busy {tot / 1e3:.3f} ms, span {span / 1e3:.3f} ms, {len(ops)} ops / {per} kernels")
    for k, g in sorted(groups.items(), key=lambda kv: -kv[1]["us"]):
        tf = g["flops"] / (g["us"] * 1e-6) / 1e12 if g["flops"] else None
        res["groups"][k] = {"ms": round(g["us"] / 1e3, 4), "launches": g["n"], "TFLOP/s": tf and round(tf, 1)}
        print(f'{g["us"] / 1e3:8.3f} ms x{g["n"]:3d} {"" if tf is None else f"{tf:6.1f} TF"}  {k}')
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        analyse(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
