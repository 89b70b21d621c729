#!/usr/bin/env python3
"""Summarise a tools/session_ab_configs.sh run: ms per call per config, A vs B runs."""
import json
import sys
from collections import defaultdict
from pathlib import Path

res = defaultdict(lambda: defaultdict(list))
for p in sorted(Path(sys.argv[1]).glob("[AB]*.out")):
    for line in p.read_text().splitlines():
        try:
            d = json.loads(line)
        except ValueError:
            continue
        if "config" in d:
            res[d["config"]][p.stem[0]].append(d.get("ms_per_call", d.get("ms")))
for cfg, v in res.items():
    print(f"{cfg:50s} A {v['A']}  B {v['B']}")
