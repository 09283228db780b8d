"""Summarise a rocprofv3 --kernel-trace CSV of bench.py into per-kernel device time per step.

bench.py runs (in order) an eager warm-up pass, a serial per-op profile pass (every launch on
one stream), then the graph warm-up / timed replays (several streams, kernels overlap, so their
rocprof durations include contention). This script finds the serial pass (the longest window
of libkrrn_hip kernels with no overlap) and reports each kernel's isolated duration there, plus the
wall-clock of each graph replay window.

usage: python profiles/kernel_trace_summary.py <run_kernel_trace.csv> [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    if name.startswith("Cijk"):
        return "hipblaslt_gemm_f32"
    m = re.search(r"(conv_gemm_f32_kernel<[^>]*>|splitk_epilogue_kernel|\w+_kernel(<[^>]*>)?|__amd_\w+)", name)
    return m.group(1) if m else name[:60]


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Queue_Id"]))
                 for r in rows if "anonymous namespace" in r["Kernel_Name"] or r["Kernel_Name"].startswith("Cijk")),
                key=lambda x: x[0])
    # mark kernels that overlap any other kernel (by more than TOL ns: back-to-back kernels of
    # one stream can show sub-microsecond timestamp overlap on a fast box)
    TOL = 2000
    iso = []
    end_max = -1
    for i, (s, e, n, q) in enumerate(ks):
        ov = s < end_max - TOL or (i + 1 < len(ks) and ks[i + 1][0] < e - TOL)
        iso.append(not ov)
        end_max = max(end_max, e)
    # serial pass = longest run of consecutive isolated kernels
    best, cur, start = (0, 0), 0, 0
    for i, ok in enumerate(iso):
        if ok:
            if cur == 0:
                start = i
            cur += 1
            if cur > best[1] - best[0]:
                best = (start, i + 1)
        else:
            cur = 0
    seg = ks[best[0]:best[1]]
    # crop the window to whole forwards: from the first forward's opening kernel (one
    # nchw_to_nhwc launch opens every forward plan) to the last step's closing kernel (the rng
    # advance ends every bench step; pnp_refine the forward + pose plan): a window that opens or
    # closes mid-forward would otherwise count a partial forward as a whole one (round-3 summary:
    # 3 "forwards" for ~2.1 steps of kernels)
    heads = [i for i, k in enumerate(seg) if k[2] == "nchw_to_nhwc_kernel"]
    for tail_name in ("advance_kernel", "pnp_refine_kernel", "tbase_tail_kernel"):
        tails = [i for i, k in enumerate(seg) if k[2] == tail_name]
        if heads and tails and tails[-1] > heads[0]:
            last = tails[-1]
            nfw = sum(1 for i in heads if i <= last)
            seg = seg[heads[0]:last + 1]
            break
    else:
        nfw = max(1, len(heads))
    per = defaultdict(lambda: [0.0, 0])
    for s, e, n, q in seg:
        per[n][0] += (e - s) / 1e3
        per[n][1] += 1
    tot = sum(v[0] for v in per.values())
    nsteps = max(1, nfw)
    res = {"serial_pass_kernels": len(seg), "serial_pass_busy_us": round(tot, 1), "forwards_in_window": nsteps,
           "busy_us_per_forward": round(tot / nsteps, 1),
           "serial_pass_span_us": round((seg[-1][1] - seg[0][0]) / 1e3, 1) if seg else 0,
           "kernels": {k: {"us": round(v[0], 1), "launches": v[1], "avg_us": round(v[0] / v[1], 2),
                           "us_per_forward": round(v[0] / nsteps, 1), "launches_per_forward": round(v[1] / nsteps, 2)}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    print(f"serial pass: {len(seg)} kernels, busy {tot / 1e3:.2f} ms, span {res['serial_pass_span_us'] / 1e3:.2f} ms, "
          f"{nsteps} forwards: {tot / nsteps / 1e3:.2f} ms busy per forward")
    for k, v in list(res["kernels"].items())[:40]:
        print(f"{v['us_per_forward'] / 1e3:8.3f} ms/fwd x{v['launches_per_forward']:7.2f} avg {v['avg_us']:9.2f} us  {k}")
    return res


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
