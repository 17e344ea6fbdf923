#!/usr/bin/env python3
"""Per-kernel HBM traffic and duration of one profiled command.

    python tools/pmc_kernels.py <dir> <out.json> --cells N [--alg kernel=bytes_per_cell ...]

<dir> holds the CSVs of three rocprofv3 runs of the same command (separate
passes, as MI355X_MICROARCH.md prescribes): fetch* (--pmc FETCH_SIZE),
write* (--pmc WRITE_SIZE) and trace* (--kernel-trace --stats).  Bytes per
launch = FETCH_SIZE (KB) x 1024 x 2 (gfx950 tallies 128-B requests at 64 B)
+ WRITE_SIZE (KB) x 1024, averaged over the kernel's launches.  With
--alg NAME=B, the kernel's algorithmic minimum is B bytes per cell x cells,
and the JSON gives traffic / minimum and minimum / duration / 8 TB/s.
"""
import argparse
import csv
import glob
import json
import os

PEAK = 8.0e12


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n.split("::")[-1] if "<" not in n else n.split("misor::")[-1]


def counters(d, prefix):
    out = {}
    for path in glob.glob(os.path.join(d, "**", prefix + "*counter_collection.csv"),
                          recursive=True):
        for r in csv.DictReader(open(path)):
            out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--cells", type=float, required=True)
    ap.add_argument("--alg", action="append", default=[],
                    help="kernel=algorithmic bytes per cell (read + write)")
    a = ap.parse_args()
    fetch = counters(a.dir, "fetch")
    write = counters(a.dir, "write")
    dur = {}
    for path in glob.glob(os.path.join(a.dir, "**", "trace*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            dur[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) * 1e-9)
    alg = dict((k, float(v)) for k, v in (s.split("=") for s in a.alg))
    res = {}
    for k in sorted(set(fetch) & set(write)):
        rd = fetch[k] * 1024 * 2
        wr = write[k] * 1024
        e = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
        if k in dur:
            e["launches"], e["avg_s"] = dur[k]
            e["actual_GBs"] = (rd + wr) / e["avg_s"] / 1e9
        if k in alg:
            m = alg[k] * a.cells
            e["alg_bytes_per_cell"] = alg[k]
            e["alg_bytes"] = m
            e["traffic_ratio"] = (rd + wr) / m
            if "avg_s" in e:
                e["alg_GBs"] = m / e["avg_s"] / 1e9
                e["frac"] = m / e["avg_s"] / PEAK
        res[k] = e
    json.dump({"cells": a.cells, "peak_GBs": PEAK / 1e9, "kernels": res}, open(a.out, "w"),
              indent=1)
    for k, e in res.items():
        if "frac" in e:
            print("%-28s %8.3f ms  traffic %.3fx  %.2f TB/s alg  frac %.3f" % (
                k, e["avg_s"] * 1e3, e["traffic_ratio"], e["alg_GBs"] / 1e3, e["frac"]))


if __name__ == "__main__":
    main()
