#!/usr/bin/env python3
"""Summarise a tools/pmc_ledger.sh run: per mode (hbm, l2, read), the mean per-dispatch value of
every counter for the measured kernel (crc32_uniform4k_kernel / stream_read_kernel), the per-wave
quad-cycle split (ACTIVE_INST_ANY + WAIT_ANY + WAIT_INST_ANY = WAVE_CYCLES), LDS array cycles per
CU and per tile, and the event-timed launch time of each mode.

  python tools/summarize_ledger.py gpurun_out/<tag> > profiles/r04/<name>.json
  python tools/summarize_ledger.py gpurun_out/<tag> list,ordered,alias,probe4,probe4o \
      crc32_small_kernel,slot_list_read          (LEDGER=small: the slot-list drain, r05)
"""
import collections
import csv
import json
import sys
from pathlib import Path

CUS, TILES = 256, 32768  # config B: 65,536 messages = 32,768 tiles of 8 KiB per launch


KERNELS = ("uniform4k", "stream_read")


def mode_counters(root: Path, mode: str) -> dict:
    tot, n = collections.defaultdict(float), collections.Counter()
    for d in sorted(root.glob(f"{mode}_p*")):
        f = d / "run_counter_collection.csv"
        if not f.exists():
            continue
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in KERNELS):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    return {c: tot[c] / n[c] for c in sorted(tot)}


def main():
    global KERNELS
    root = Path(sys.argv[1])
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["hbm", "l2", "read"]
    if len(sys.argv) > 3:
        KERNELS = tuple(sys.argv[3].split(","))
    out = {"source": str(root), "kernels": list(KERNELS), "modes": {}}
    for mode in modes:
        c = mode_counters(root, mode)
        t = root / f"{mode}_t.json"
        entry = {"timing": json.loads(t.read_text()) if t.exists() else None, "counters": c}
        waves = c.get("SQ_WAVES")
        if waves:
            entry["per_wave_quad_cycles"] = {k: round(c[k] / waves) for k in
                                             ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                              "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS")
                                             if k in c}
            entry["per_wave_insts"] = {k: round(c[k] / waves) for k in
                                       ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD")
                                       if k in c}
        if "SQ_LDS_IDX_ACTIVE" in c:
            entry["lds_cycles_per_cu"] = round(c["SQ_LDS_IDX_ACTIVE"] / CUS)
            entry["lds_conflict_cycles_per_cu"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / CUS)
            entry["lds_cycles_per_tile"] = round(c["SQ_LDS_IDX_ACTIVE"] / TILES, 1)
            entry["lds_conflict_cycles_per_tile"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / TILES, 1)
        if "GRBM_GUI_ACTIVE" in c:
            entry["gui_active_cycles_per_xcd"] = round(c["GRBM_GUI_ACTIVE"] / 8)
        out["modes"][mode] = entry
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
