"""HRNet-phase idle time per stream in the last graph-replayed step of a rocprofv3 kernel trace:
the window from the first to the last conv_small launch of the step; per queue, the span between
its first and last kernel in the window minus the time a kernel of that queue was running.

usage: python3 profiles/hrnet_waits.py run_kernel_trace.csv [...]"""
import csv
import sys


def step_rows(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    starts = [i for i, k in enumerate(ks) if "randperm_multi" in k[2]]
    spans = [(ks[b][0] - ks[a][0], a, b) for a, b in zip(starts, starts[1:])]
    fast = min(sp for sp, _, _ in spans)
    lo, hi = [(a, b) for sp, a, b in spans if sp <= 1.2 * fast][-1]
    return ks[lo:hi]


for path in sys.argv[1:]:
    step = step_rows(path)
    small = [k for k in step if "conv_small" in k[2]]
    w0, w1 = small[0][0], max(k[1] for k in small)
    print(f"{path}: step {(max(k[1] for k in step) - step[0][0]) / 1e3:.0f} us, HRNet window {(w1 - w0) / 1e3:.0f} us")
    for q in sorted({k[3] for k in step}):
        ks = [k for k in step if k[3] == q and k[1] > w0 and k[0] < w1]
        if len(ks) < 5:
            continue
        busy, cs, ce = 0, None, None
        for s, e, *_ in ks:
            s, e = max(s, w0), min(e, w1)
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        span = min(max(k[1] for k in ks), w1) - max(ks[0][0], w0)
        print(f"  queue {q}: {len(ks)} kernels, span {span / 1e3:.0f} us, busy {busy / 1e3:.0f} us, "
              f"idle {(span - busy) / 1e3:.0f} us")
