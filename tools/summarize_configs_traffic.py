#!/usr/bin/env python3
"""Summarise tools/pmc_configs.sh: per configuration, the HBM bytes of one C-ABI call (every
dispatch of the call's kernels -- setup kernels excluded by name -- summed and divided by the
calls made), FETCH_SIZE doubled per MI355X_MICROARCH.md "HBM" (gfx950 tallies a wide 16-B/lane
read's 128-B requests at 64 B), WRITE_SIZE as measured; against the call's algorithmic bytes.

  python tools/summarize_configs_traffic.py gpurun_out/<tag> [profiles/traffic_configs.json] [--merge]
(--merge: keep the file's other configurations; each entry records its own source.)
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

SETUP = ("synth_fill", "rocclr", "at::native", "elementwise", "reduce_kernel")


def per_call(d: Path, counter: str, calls: int):
    f = d / "run_counter_collection.csv"
    if not f.exists():
        return None, {}
    tot, kern = 0.0, defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter or any(x in r["Kernel_Name"] for x in SETUP):
            continue
        v = float(r["Counter_Value"])
        tot += v
        kern[r["Kernel_Name"].split("(")[0].replace("void ", "")] += v
    return tot / calls, {k: round(v / calls, 1) for k, v in kern.items()}


def main():
    args = [a for a in sys.argv[1:] if a != "--merge"]
    root = Path(args[0])
    out_path = Path(args[1]) if len(args) > 1 else Path(__file__).resolve().parent.parent / "profiles" / \
        "traffic_configs.json"
    src = str(root).replace(str(Path(__file__).resolve().parent.parent) + "/", "")
    res = {"source": src,
           "correction": "HBM bytes per call = (FETCH_SIZE x 2 + WRITE_SIZE) x 1024, every dispatch of the call's "
                         "kernels (MI355X_MICROARCH.md HBM; separate PMC passes)", "configs": {}}
    if "--merge" in sys.argv and out_path.exists():
        old = json.loads(out_path.read_text())
        res["source"] = old.get("source", src)
        for k, v in old.get("configs", {}).items():
            v.setdefault("source", res["source"])
            res["configs"][k] = v
    for j in sorted(root.glob("*_FETCH_SIZE.json")):
        name = j.name[:-len("_FETCH_SIZE.json")]
        try:
            meta = json.loads(j.read_text().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        calls, alg = meta["calls"], meta["algorithmic_bytes_per_call"]
        f_kib, f_k = per_call(root / f"{name}_FETCH_SIZE", "FETCH_SIZE", calls)
        w_kib, _ = per_call(root / f"{name}_WRITE_SIZE", "WRITE_SIZE", calls)
        if f_kib is None:
            continue
        hbm = (2 * f_kib + (w_kib or 0.0)) * 1024
        res["configs"][name] = {"hbm_bytes_per_call": round(hbm), "hbm_read_bytes_per_call": round(2 * f_kib * 1024),
                                "write_bytes_per_call": round((w_kib or 0.0) * 1024),
                                "algorithmic_bytes_per_call": alg, "ratio": round(hbm / alg, 4), "source": src,
                                "fetch_kib_per_call_by_kernel": f_k}
    out_path.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: v["ratio"] for k, v in res["configs"].items()}))
    return res


if __name__ == "__main__":
    main()
