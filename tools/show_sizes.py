#!/usr/bin/env python3
"""Tabulates tools/small_sizes.py result files (investigation helper): one row per message size,
one column per file, µs per call.  python tools/show_sizes.py <file.jsonl> ..."""
import json
import sys
from pathlib import Path

cols, rows = [], {}
for f in sys.argv[1:]:
    name = Path(f).stem
    cols.append(name)
    for line in open(f):
        d = json.loads(line)
        key = str(d.get("message", d.get("length", d.get("ragged_max"))))
        rows.setdefault(key, {})[name] = d["us_per_call"] if d.get("all_pass", True) else f"{d['us_per_call']}!"
print("size".ljust(10) + "".join(c[:22].rjust(24) for c in cols))
for k, v in rows.items():
    print(k.ljust(10) + "".join(str(v.get(c, "")).rjust(24) for c in cols))
