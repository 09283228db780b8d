"""Timeline of the last graph-replayed step from a rocprofv3 kernel trace: wall span, busy
union, per-kernel start/end offsets (us) and the number of concurrently running kernels."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])) * int(r["Grid_Size_Y"]), r["Queue_Id"]) for r in rows]
ks.sort()
# step = from one randperm_multi launch (the forward's pool draws) to the next; the graph-replayed
# steps come before bench.py's serial profiling pass, so take the last step whose span is within
# 1.2x of the shortest one
starts = [i for i, k in enumerate(ks) if "randperm_multi" in k[2]]
spans = [(ks[b][0] - ks[a][0], a, b) for a, b in zip(starts, starts[1:])]
fast = min(sp for sp, _, _ in spans)
lo, hi = [(a, b) for sp, a, b in spans if sp <= 1.2 * fast][-1]
step = ks[lo:hi]
t0 = step[0][0]
t1 = max(k[1] for k in step)
busy, cur_s, cur_e = 0, None, None
for s, e, *_ in step:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"kernels {len(step)} wall {(t1 - t0) / 1e3:.1f} us busy {busy / 1e3:.1f} us sum {sum(e - s for s, e, *_ in step) / 1e3:.1f} us")
mode = sys.argv[2] if len(sys.argv) > 2 else "all"
for s, e, n, g, q in step:
    conc = sum(1 for s2, e2, *_ in step if s2 < e and e2 > s) - 1
    short = n.replace("void ", "").replace("(anonymous namespace)::", "")[:70]
    if mode == "all" or (e - s) > 20000:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} wg={g:6d} c={conc} {short}")
