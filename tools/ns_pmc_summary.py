#!/usr/bin/env python3
"""HBM bytes per launch of the NS config-5 streaming kernels from separate
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu/r5_v.sh), with the
gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE KB x 1024 x 2 + WRITE_SIZE
KB x 1024), against each kernel's algorithmic bytes (40 B per cell: fg_rhs
reads u, v and writes f, g, rhs; adapt_absmax reads f, g, p and writes u, v).

    python tools/ns_pmc_summary.py gpurun_out/r5v profiles/r05_pmc_ns16384_nt.json --size 16384
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(d, prefix, counter):
    acc = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", prefix + "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            for k in ("fg_rhs_kernel", "adapt_absmax_kernel"):
                if k in name:
                    acc[k].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=16384)
    a = ap.parse_args()
    fetch = per_kernel(a.dir, "fetch", "FETCH_SIZE")
    write = per_kernel(a.dir, "write", "WRITE_SIZE")
    cells = a.size * a.size
    res = {"size": a.size, "algorithmic_bytes_per_launch": 40 * cells, "kernels": {}}
    for k in sorted(fetch):
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write[k]) / len(write[k])
        b = f * 1024 * 2 + w * 1024
        res["kernels"][k] = {"launches": len(fetch[k]), "fetch_size_kb_raw": f,
                             "write_size_kb": w, "read_bytes_corrected": f * 2048,
                             "write_bytes": w * 1024, "bytes_per_launch": b,
                             "ratio_to_algorithmic": b / (40 * cells)}
    res["note"] = ("separate rocprofv3 --pmc passes of bench.py --workload ns; FETCH_SIZE x1024 x2 "
                   "(gfx950: 128-B requests tallied at 64 B) + WRITE_SIZE x1024")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main()
