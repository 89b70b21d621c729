#!/usr/bin/env python3
"""rocprofv3's SQLite output (run_results.db, the default format) -> the kernel-trace CSV columns
the other tools read (Kernel_Name, Start_Timestamp, End_Timestamp).

  python tools/rocpd_to_csv.py gpurun_out/<tag>/prof/run_results.db > kernel_trace.csv
"""
import csv
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    rows = db.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                      "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    w = csv.writer(sys.stdout)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
    for name, start, end in rows:
        w.writerow([name, start, end])


if __name__ == "__main__":
    main(sys.argv[1])
