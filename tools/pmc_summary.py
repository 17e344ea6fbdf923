#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_bench.sh into profiles/<name>.json.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/r01_pmc_tb7_32768.json \
        --size 32768 --iters 7 [--kernel rb_tb_kernel]

HBM bytes per launch, corrected as MI355X_MICROARCH.md prescribes for gfx950:
FETCH_SIZE (KB) x 1024 x 2 (it tallies 128-B requests at 64 B) + WRITE_SIZE (KB)
x 1024, averaged over the launches of the kernel.  bench.py reads
`bytes_per_launch` back as roofline.traffic for the same size / ranks / T.
"""
import argparse
import csv
import glob
import json
import os


def rows(d, prefix, kernel):
    out = {}
    for path in glob.glob(os.path.join(d, "**", prefix + "*counter_collection.csv"),
                          recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                out.setdefault(r["Counter_Name"], []).append(
                    (r["Kernel_Name"], int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return out


def mean(v):
    return sum(x[2] for x in v) / len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--iters", type=int, required=True)
    ap.add_argument("--kernel", default=None,
                    help="kernel name substring (default: rb_tb_kernel<ITERS, -- only the "
                         "full passes, not the warm-up or remainder instantiations)")
    ap.add_argument("--rows", type=int, default=0)
    a = ap.parse_args()
    if a.kernel is None:
        a.kernel = "rb_tb_kernel<%d," % a.iters
    f = rows(a.dir, "fetch", a.kernel)
    w = rows(a.dir, "write", a.kernel)
    s = rows(a.dir, "sq", a.kernel)
    # full-iteration launches only (a capped solve's last pass may run fewer)
    fetch = f["FETCH_SIZE"]
    write = w["WRITE_SIZE"]
    rd = mean(fetch) * 1024 * 2
    wr = mean(write) * 1024
    cells = float(a.size) * a.size / a.nranks
    hbm_min = 24 * cells
    out = {
        "size": a.size, "nranks": a.nranks, "iters_per_pass": a.iters,
        "kernel": fetch[0][0].split("(")[0].replace("void ", ""),
        "rows_per_block": a.rows or None, "launches": len(fetch),
        "fetch_size_kb_raw": mean(fetch), "write_size_kb": mean(write),
        "read_bytes_corrected": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
        "hbm_minimum_bytes_per_launch": hbm_min,
        "algorithmic_bytes_per_launch": hbm_min * a.iters,
        "ratio_to_hbm_minimum": (rd + wr) / hbm_min,
    }
    if s:
        cyc = mean(s["SQ_WAVE_CYCLES"]) if "SQ_WAVE_CYCLES" in s else None
        sq = {}
        for k, name in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst_any"),
                        ("SQ_ACTIVE_INST_ANY", "active_inst_any"),
                        ("SQ_ACTIVE_INST_VALU", "active_inst_valu")):
            if cyc and k in s:
                sq[name] = round(mean(s[k]) / cyc, 3)
        if "SQ_INSTS_VALU" in s:
            sq["valu_insts"] = mean(s["SQ_INSTS_VALU"])
        out["sq"] = sq
    out["note"] = ("one launch = %d solveRB iterations (temporally blocked); FETCH_SIZE x1024 x2 "
                   "(gfx950 correction, MI355X_MICROARCH.md HBM) + WRITE_SIZE x1024; separate "
                   "rocprofv3 --pmc passes (tools/profile_bench.sh); the HBM minimum of a launch "
                   "is 24 B x cells (p, rhs read once, p written once)" % a.iters)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
