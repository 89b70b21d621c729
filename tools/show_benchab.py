#!/usr/bin/env python3
"""Summarise a tools/session_benchab.sh run: per library, bench.py's us per step."""
import json
import sys
from collections import defaultdict
from pathlib import Path

res = defaultdict(list)
for p in sorted(Path(sys.argv[1]).glob("b_*.out")):
    name = p.stem[2:].rsplit("_", 1)[0]
    lines = [ln for ln in p.read_text().splitlines() if ln.startswith("{")]
    if lines:
        d = json.loads(lines[-1])
        res[name].append(round(d["ms_per_step"] * 1e3, 2) if d["ms_per_step"] > 0.1 else
                         round(2**28 * d["n_gpus"] / (d["value"] * 2**30) * 1e6, 2))
for name, v in sorted(res.items()):
    print(name, v, "median", sorted(v)[len(v) // 2])
