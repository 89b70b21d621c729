#!/usr/bin/env python3
"""Summarise a tools/session_slotab.sh run: per variant, per library, the median over rounds
of slot_gap.py's median us per call.   python tools/show_slotab.py gpurun_out/<tag>"""
import collections
import glob
import json
import statistics
import sys

res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{sys.argv[1]}/g_*.out")):
    lib = f.split("/")[-1][2:].rsplit("_", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            res[d["variant"]][lib].append(d["median_us"])
for v, libs in res.items():
    print(v, {k: (round(statistics.median(x), 2), x) for k, x in libs.items()})
