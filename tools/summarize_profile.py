#!/usr/bin/env python3
"""Summarise a GPU session's rocprofv3 output into profiles/<tag>/.

  python tools/summarize_profile.py <session-dir> <tag>

Reads <session-dir>/prof/run_kernel_stats.csv (--kernel-trace --stats) and the separate
PMC passes <session-dir>/pmc_FETCH_SIZE/, pmc_WRITE_SIZE/ (one counter per pass), and writes
  profiles/<tag>/kernel_stats.csv        copy of the rocprofv3 summary
  profiles/<tag>/summary.md              per-kernel averages + HBM traffic per launch
  profiles/traffic_uniform4k.json        read by bench.py (roofline.traffic)

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B stores and uncalibrated for our 4-B result stores
(4 B per message, 0.1 % of the traffic), reported as measured.
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def per_dispatch(pmc_dir: Path, counter: str):
    f = pmc_dir / "run_counter_collection.csv"
    if not f.exists():
        return {}
    vals = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        key = r["Dispatch_Id"]
        vals[key] += float(r["Counter_Value"])
        names[key] = r["Kernel_Name"]
    by_kernel = defaultdict(list)
    for k, v in vals.items():
        by_kernel[names[k]].append(v)
    return by_kernel


def timed_launches(trace: Path, name_part: str, k: int):
    """(average duration us, start-to-start interval us, n) over the last k dispatches of
    the kernel whose name contains name_part, from a --kernel-trace CSV."""
    if not trace.exists():
        return None
    rows = [r for r in csv.DictReader(open(trace)) if name_part in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = rows[-k:]
    if len(last) < 2:
        return None
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last]
    span = int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])
    return sum(durs) / len(durs) / 1e3, span / len(last) / 1e3, len(last), sorted(d / 1e3 for d in durs)


def main():
    sess, tag = Path(sys.argv[1]), sys.argv[2]
    out = ROOT / "profiles" / tag
    out.mkdir(parents=True, exist_ok=True)
    # profsel: rocprofv3 --selected-regions around bench.py --roctx-region (exactly the K timed
    # launches); prof: the whole run (settle and warm-up launches included)
    pdir = next((sess / d for d in ("profsel", "prof") if (sess / d / "run_kernel_stats.csv").exists()), sess / "prof")
    stats = pdir / "run_kernel_stats.csv"
    rows = list(csv.DictReader(open(stats))) if stats.exists() else []
    if stats.exists():
        shutil.copy(stats, out / "kernel_stats.csv")
    fetch = per_dispatch(sess / "pmc_FETCH_SIZE", "FETCH_SIZE")
    write = per_dispatch(sess / "pmc_WRITE_SIZE", "WRITE_SIZE")
    lines = [f"# rocprofv3 summary ({tag})", "",
             f"Source: `{sess}` (rocprofv3 --kernel-trace --stats"
             + (" --selected-regions: only bench.py's timed region, bracketed by roctxProfilerResume/Pause"
                if pdir.name == "profsel" else "") + "; PMC FETCH_SIZE and WRITE_SIZE in separate passes).",
             "", "| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} |")
    # the headline kernel (not its slot variant crc32_uniform4k_kernel<512, true, false>)
    timed = timed_launches(pdir / "run_kernel_trace.csv", "crc32_uniform4k_kernel<512, false, false>", 1000)
    if timed:
        avg, per, n, sd = timed
        where = (f"bench.py's timed region = the {n} dispatches recorded (rocprofv3 --selected-regions)"
                 if pdir.name == "profsel" else
                 f"bench.py's timed region = the last {n} dispatches of the uniform kernel (the earlier "
                 "ones are the settle and warm-up launches, which include the power-management ramp)")
        lines += ["", where + ": "
                  f"average kernel duration {avg:.2f} us, dispatch-to-dispatch interval {per:.2f} us "
                  f"(= {65536 * 4096 / per / 1e3:.0f} GB/s of payload; bench.py's roofline.achieved uses the "
                  "HIP-event span of the same region / K). Per-launch durations: median "
                  f"{sd[len(sd) // 2]:.2f} us, best {sd[0]:.2f}, 10th percentile {sd[len(sd) // 10]:.2f}, "
                  f"90th {sd[(9 * len(sd)) // 10]:.2f}, worst {sd[-1]:.2f}."]
    lines += ["", "| kernel | dispatches | FETCH_SIZE KiB/launch (raw) | HBM read bytes/launch (x2, gfx950) | "
              "WRITE_SIZE KiB/launch |", "|---|---|---|---|---|"]
    traffic = {}
    for name, v in fetch.items():
        # drop the first dispatches (warm-up) when there are enough
        vv = v[2:] if len(v) > 4 else v
        f_kib = sum(vv) / len(vv)
        w = write.get(name, [])
        ww = w[2:] if len(w) > 4 else w
        w_kib = sum(ww) / len(ww) if ww else float("nan")
        rd = 2 * f_kib * 1024
        lines.append(f"| `{name[:90]}` | {len(v)} | {f_kib:.0f} | {rd:.4g} | {w_kib:.0f} |")
        if "crc32_uniform4k_kernel<512, false, false>" in name:
            traffic = {"kernel": name, "fetch_size_kib_per_launch": f_kib, "write_size_kib_per_launch": w_kib,
                       "hbm_bytes_per_launch": rd + (w_kib * 1024 if w_kib == w_kib else 0.0),
                       "hbm_read_bytes_per_launch": rd, "algorithmic_bytes_per_launch": 65536 * 4096,
                       "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount, MI355X_MICROARCH.md HBM)",
                       "source": f"profiles/{tag}"}
    # HBM bytes per launch against the algorithmic bytes, for the launches whose size is fixed
    # in bench.py's PMC passes: config B (65,536 x 4 KiB) and config S (65,536 slots: 4 KiB
    # payload + the 64-B prefix line each)
    algo = {"crc32_uniform4k_kernel<512, false, false>": ("B", 65536 * 4096),
            "crc32_uniform4k_kernel<512, true, false>": ("S", 65536 * (4096 + 64))}
    ratio_lines = []
    for name, v in fetch.items():
        for part, (cfg, nbytes) in algo.items():
            if part in name:
                vv = v[2:] if len(v) > 4 else v
                w = write.get(name, [])
                ww = w[2:] if len(w) > 4 else w
                rd = 2 * sum(vv) / len(vv) * 1024
                wr = sum(ww) / len(ww) * 1024 if ww else 0.0
                ratio_lines.append(f"| `{part}` (config {cfg}) | {nbytes:.4g} | {rd + wr:.4g} | {(rd + wr) / nbytes:.3f} |")
    # configs C and D (bench.py's default configs; the ragged kernel's dispatches split by size:
    # C reads ~118 GB per call, D 17 GB) and D through the uniform API (the long-message kernel).
    # FETCH_SIZE x 2 is the streaming-read calibration; for C's many partial last lines it
    # may overstate the bytes a little.
    big = {"C": (117844131581, lambda v: v * 2048 > 60e9), "D": (256 * (64 << 20), lambda v: v * 2048 <= 60e9)}
    for name, v in fetch.items():
        if "crc32_ragged_kernel" in name:
            for cfg, (nbytes, sel) in big.items():
                vv = [x for x in v if sel(x)]
                if vv:
                    rd = 2 * sum(vv) / len(vv) * 1024
                    ratio_lines.append(f"| `crc32_ragged_kernel<512>` (config {cfg}, {len(vv)} calls) | {nbytes:.4g} | "
                                       f"{rd:.4g} (read) | {rd / nbytes:.3f} |")
        elif "crc32_long_kernel" in name and v:
            rd = 2 * sum(v) / len(v) * 1024
            nbytes = 256 * (64 << 20)
            ratio_lines.append(f"| `crc32_long_kernel<512>` (config D, uniform API, {len(v)} calls) | {nbytes:.4g} | "
                               f"{rd:.4g} (read) | {rd / nbytes:.3f} |")
    if ratio_lines:
        lines += ["", "| kernel | algorithmic bytes / launch | HBM bytes / launch (read x2 + write) | ratio |",
                  "|---|---|---|---|"] + ratio_lines
    (out / "summary.md").write_text("\n".join(lines) + "\n")
    if traffic:
        (ROOT / "profiles" / "traffic_uniform4k.json").write_text(json.dumps(traffic, indent=1) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
