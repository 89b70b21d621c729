#!/usr/bin/env python3
"""Per-call breakdown of the ragged / long paths from a rocprofv3 kernel trace.

  python tools/prep_breakdown.py gpurun_out/<tag>/prof/run_kernel_trace.csv

Groups the trace into calls (a call starts at crc32_ragged_count_scan_kernel or at
crc32_long_kernel), classifies each call by its main kernel's duration (> 10 ms: config C,
else config D) and prints the median duration of every kernel and of everything but the
main kernel (prep + combine) per class, in microseconds.
"""
import collections
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "subspace_amd" not in name:
            continue
        short = name.split("(")[0].replace("void ", "").replace("subspace_amd::", "")
        if "count_scan" in name or "count_desc" in name or "crc32_long_kernel" in name:
            cur = collections.OrderedDict()
            calls.append(cur)
        if cur is not None:
            cur[short] = cur.get(short, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    mains = ("crc32_ragged_kernel<512>", "crc32_long_kernel<512>")
    by = collections.defaultdict(list)
    for c in calls:
        main_us = sum(c.get(m, 0.0) for m in mains)
        by[("C" if main_us > 10000 else "D") + (" (long kernel)" if mains[1] in c else "")].append(c)
    for key, cs in by.items():
        print(f"{key}: {len(cs)} calls")
        for n in cs[0]:
            v = sorted(c.get(n, 0.0) for c in cs)
            print(f"   {n:40s} {v[len(v) // 2]:10.2f}")
        prep = sorted(sum(t for n, t in c.items() if n not in mains) for c in cs)
        print(f"   {'prep + combine':40s} {prep[len(prep) // 2]:10.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
