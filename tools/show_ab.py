#!/usr/bin/env python3
"""Summarise a tools/ab_session.sh run: per library, every JSON field that holds a timing
(median_us of slot_gap variants, or the sweep's us per launch), sorted over its runs."""
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
res = defaultdict(lambda: defaultdict(list))
for f in sorted(d.glob("run*_*.jsonl")):
    lib = re.match(r"run\d+_(.+)", f.stem).group(1)
    for line in f.read_text().splitlines():
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        if "variant" in r:
            res[lib][r["variant"]].append(r["median_us"])
        else:
            for k, v in r.items():
                if isinstance(v, (int, float)) and not isinstance(v, bool) and k not in ("round", "count", "wg",
                                                                                         "order", "launches"):
                    res[lib][k].append(v)
for lib, r in sorted(res.items()):
    print(lib, json.dumps({k: sorted(x) for k, x in r.items()}))
