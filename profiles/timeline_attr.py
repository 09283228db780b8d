"""Where the graph-replayed step's wall time goes: rocprofv3 --kernel-trace of bench.py, the
timed replay window (the longest run of kernels on several queues), each instant of it shared
equally by the kernels running then (1/k each when k overlap); idle instants counted apart.
Per kernel family: attributed wall ms per step, serial (isolated-duration) ms per step, and the
mean concurrency it ran at.

usage: python profiles/timeline_attr.py run_kernel_trace.csv STEPS [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(n):
    if n.startswith("Cijk"):
        return "hipblaslt"
    m = re.search(r"(\w+_kernel(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


def main(path, steps, out=None):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Queue_Id"]))
                for r in rows)
    wins, cur, end = [], [ks[0]], ks[0][1]
    for k in ks[1:]:
        if k[0] - end > 150000:
            wins.append(cur)
            cur = [k]
        else:
            cur.append(k)
        end = max(end, k[1])
    wins.append(cur)
    multi = [w for w in wins if len(set(k[3] for k in w)) > 1]
    w = max(multi, key=len)
    t0, t1 = w[0][0], max(k[1] for k in w)
    ev = sorted([(s, 1, i) for i, (s, e, n, q) in enumerate(w)] + [(e, -1, i) for i, (s, e, n, q) in enumerate(w)])
    attr = defaultdict(float)
    serial = defaultdict(float)
    cnt = defaultdict(int)
    conc_w = defaultdict(float)
    active = set()
    idle = 0.0
    last = t0
    for t, d, i in ev:
        dt = t - last
        if dt > 0:
            if active:
                for j in active:
                    attr[w[j][2]] += dt / len(active)
                    conc_w[w[j][2]] += dt * len(active)
            else:
                idle += dt
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    for s, e, n, q in w:
        serial[n] += e - s
        cnt[n] += 1
    span = (t1 - t0) / 1e6
    res = {"window_ms": round(span, 3), "steps": steps, "ms_per_step": round(span / steps, 3),
           "idle_ms_per_step": round(idle / 1e6 / steps, 3), "kernels": {}}
    for n in sorted(attr, key=lambda n: -attr[n]):
        res["kernels"][n] = {"attributed_ms_per_step": round(attr[n] / 1e6 / steps, 4),
                             "busy_ms_per_step": round(serial[n] / 1e6 / steps, 4),
                             "launches_per_step": round(cnt[n] / steps, 2),
                             "mean_concurrency": round(conc_w[n] / max(serial[n], 1), 2)}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    print(f"window {span:.2f} ms = {steps} steps x {span / steps:.3f} ms; idle {idle / 1e6 / steps:.3f} ms/step")
    print(f"{'kernel':45s} {'attr ms':>8s} {'busy ms':>8s} {'launch':>7s} {'conc':>5s}")
    for n, v in list(res["kernels"].items())[:35]:
        print(f"{n[:45]:45s} {v['attributed_ms_per_step']:8.3f} {v['busy_ms_per_step']:8.3f} "
              f"{v['launches_per_step']:7.1f} {v['mean_concurrency']:5.2f}")
    return res


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None)
