"""Wall time of graph-replayed stages: backbone (ops[:split]), heads (split:heads_end), tail (rest)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import KRRN, make_config
from pose_estimation_amd.pipeline import BatchPipeline, _sub_plan
from pose_estimation_amd.synthetic import init_weights, make_batch
dev = torch.device("cuda", 0)
B, S, N = 64, 120, 1000
m = KRRN(cfg=make_config(num_cls=1, backbone="w18")); init_weights(m, 0); m = m.to(dev).eval()
pl = BatchPipeline(m, B, S, N, dev, parts=1, seed=3)
pl.load(make_batch(B, S, N, seed=1)); pl.run(); torch.cuda.synchronize()
pt = pl.parts[0]; kp = pt.kp
stages = {"backbone": [(_sub_plan(kp.plan, 0, kp.split), kp.env)],
          "heads": [(_sub_plan(kp.plan, kp.split, kp.heads_end), kp.env)],
          "tail": [(kp.device_perm_plan, {}), (_sub_plan(kp.plan, kp.heads_end, len(kp.plan.ops)), kp.env), (pt.pose, {})],
          "all": [(kp.device_perm_plan, {}), (kp.plan, kp.env), (pt.pose, {})]}
if os.environ.get("NOPNP"):
    from pose_estimation_amd.runtime import Plan
    tp = _sub_plan(kp.plan, kp.heads_end, len(kp.plan.ops))
    tp.ops = [o for o in tp.ops if not (o.name != "sync" and o.sid == 6) and not (o.name == "sync" and 6 in (o.src, o.dst))]
    stages["tail_nopnp"] = [(kp.device_perm_plan, {}), (tp, kp.env), (pt.pose, {})]
    pp = _sub_plan(kp.plan, kp.heads_end, len(kp.plan.ops))
    pp.ops = [o for o in pp.ops if o.name != "sync" and o.sid == 6]
    for o in pp.ops: pass
    stages["pnp_only"] = [(pp, kp.env)]
for name, plans in stages.items():
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for p, env in plans: p.run(dict(env))
    torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for p, env in plans: p.run(dict(env))
    torch.cuda.synchronize()
    for _ in range(3): g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): g.replay()
    b.record(); torch.cuda.synchronize()
    n_k = sum(len([o for o in p.ops if o.name != "sync"]) for p, _ in plans)
    print(f"{name:9s} {a.elapsed_time(b) / 20:7.3f} ms  ({n_k} launches)", flush=True)
