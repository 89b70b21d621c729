#!/usr/bin/env python3
"""Summarise a tools/session_multi.sh run: per library, the timeline medians and the
interleaved launch times (us)."""
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
libs = sorted({p.name[3:-4] for p in d.glob("tl_*.out")})
for n in libs:
    lines = (d / f"tl_{n}.out").read_text().strip().splitlines()
    m = json.loads(lines[-1])["median_over_launches"] if lines else {}
    ab = []
    for p in sorted(d.glob(f"ab_{n}_*.out")):
        for line in p.read_text().splitlines():
            ab.append(round(json.loads(line)["median_ms"] * 1e3, 2))
    print(n, "launch us:", ab, "| timeline:", {k: m.get(k) for k in
          ("fill_p50", "tile0_landed_p50", "loop_end_by_wave_in_wg", "exit_p50", "exit_max", "period")})
