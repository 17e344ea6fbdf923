#!/usr/bin/env python3
"""Print the kernel timeline of a rocprofv3 --kernel-trace CSV between two
dispatch indices (diagnostics): start / end relative to the first kernel shown
(us), duration, queue, short name; and the idle gaps of the GPU between them.

    python tools/timeline.py gpurun_out/r5m/.../trace_kernel_trace.csv [--last 80]
"""
import argparse
import csv
import glob
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=80)
    a = ap.parse_args()
    path = a.csv if a.csv.endswith(".csv") else glob.glob(a.csv + "/**/*kernel_trace.csv",
                                                            recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.last:]
    t0 = int(rows[0]["Start_Timestamp"])
    busy_end = t0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("misor::", "")
        gap = (s - busy_end) / 1e3
        print("%9.1f %9.1f %8.1f  q%-3s grid %-7s %s%s" % (
            (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, r.get("Queue_Id", ""),
            r.get("Grid_Size_X", ""), name[:60], "   <- idle %.1f us" % gap if gap > 2 else ""))
        busy_end = max(busy_end, e)


if __name__ == "__main__":
    main()
