"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate
runs, as MI355X_MICROARCH.md §rocprofv3 PMC slots requires).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half of the bytes of a
wide (16 B/lane) coalesced read, so read bytes = 2 * FETCH_SIZE KiB; WRITE_SIZE is exact for
16 B/lane stores. Both counters are in KiB.

    python profiles/pmc_traffic.py FETCH.csv WRITE.csv [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def _short(name: str) -> str:
    m = re.search(r"conv_gemm_f32_kernel<(\d+), (\d+), (\d+), \d+, (true|false)>", name)
    if m:
        return f"conv_gemm_f32<{m.group(1)},{m.group(2)},{m.group(3)}>" + (",nchw" if m.group(4) == "true" else "")
    m = re.search(r"conv_group_kernel<(\d+), (\d+), (\d+), \d+>", name)
    if m:
        return f"conv_group<{m.group(1)},{m.group(2)},{m.group(3)}>"
    if re.search(r"wino_f43_x3_kernel<(true|[1-4])>", name):
        return "wino_f43_x3_head"
    if "wino_f43_x3" in name:
        return "wino_f43_x3"
    if "wino_f23_x3_kernel<true>" in name:
        return "wino_f23_x3_head"
    if "wino_f23_x3" in name:
        return "wino_f23_x3"
    if "wino_f23" in name:
        return "wino_f23<32,32,16>"
    m = re.search(r"conv3x3_small_kernel<(\d+), (\d+)>", name)
    if m:
        return f"conv3x3_small<{m.group(1)},{m.group(2)}>"
    if name.startswith("Cijk"):
        return "hipblaslt_gemm_f32"
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            per[_short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        fr, wr = fetch.get(k, []), write.get(k, [])
        if not fr or not wr:
            continue
        rd = 2.0 * sum(fr) / len(fr) * 1024.0
        wb = sum(wr) / len(wr) * 1024.0
        out[k] = {"launches": len(fr), "read_bytes_per_launch": rd, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": rd + wb}
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(js)
    print(js)


if __name__ == "__main__":
    main()
