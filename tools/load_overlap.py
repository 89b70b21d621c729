#!/usr/bin/env python3
"""List the vector loads whose destination VGPRs overlap their own address VGPRs, per kernel,
in a HIP source's gfx950 device code (investigation tool; r05: such a load in the slot-list
drain's tile loop -- `global_load_dwordx4 v[56:59], v[56:57], off offset:64`, the address dead
after the tile's last load and reused as its destination -- measured 8 us slower per
65,536-slot call than the same loop with a separate address pair, tools/ledger_small.py).

  python tools/load_overlap.py subspace_amd/csrc/crc_small.hip [--all] [-D...]
(16-B loads only unless --all; exit status 1 when any load overlaps.)
"""
import re
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

LOAD = re.compile(r"(global|buffer|flat)_load_dword\w*\s+v\[(\d+):(\d+)\],\s*(?:v\[(\d+):(\d+)\]|v(\d+))")


def overlaps(src, flags=(), every=False):
    """{kernel: (overlapping loads, loads)} for the gfx950 device code of `src` (16-B loads only
    unless every)."""
    with tempfile.TemporaryDirectory() as d:
        co = Path(d) / "k.co"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "--no-gpu-bundle-output", *flags, "-c", str(src), "-o", str(co)], check=True)
        dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", str(co)], check=True,
                             capture_output=True, text=True).stdout
    kernel, loads, over = None, Counter(), Counter()
    for line in dis.splitlines():
        if re.match(r"^[0-9a-f]+ <", line):
            kernel = line.split("<", 1)[1].rstrip(">:")
        m = LOAD.search(line)
        if m and kernel and ("x4" in line or every):
            d0, d1 = int(m.group(2)), int(m.group(3))
            a0 = int(m.group(4) or m.group(6))
            a1 = int(m.group(5) or m.group(6))
            loads[kernel] += 1
            if not (a1 < d0 or a0 > d1):
                over[kernel] += 1
    return {k: (over[k], loads[k]) for k in loads}


def main():
    every = "--all" in sys.argv  # also single-dword and 64-bit loads (records, prefix words)
    src, flags = sys.argv[1], [f for f in sys.argv[2:] if f != "--all"]
    res = overlaps(src, flags, every)
    for k, (o, n) in res.items():
        print(f"{o:4d} of {n:4d} loads overlap  {k}")
    return 1 if any(o for o, _ in res.values()) else 0


if __name__ == "__main__":
    sys.exit(main())
