#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_bench.sh into profiles/<name>.json.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/r01_pmc_tb7_32768.json \
        --size 32768 --iters 7 [--kernel rb_tb_kernel]
    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/r03_pmc_tb{T}_32768.json \
        --size 32768 --iters all      (one summary per pass length found)

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
import re


def rows(d, prefix, kernel):
    out = {}
    for path in glob.glob(os.path.join(d, "**", prefix + "*counter_collection.csv"),
                          recursive=True):
        for r in csv.DictReader(open(path)):
            if re.search(kernel, r["Kernel_Name"]):
                out.setdefault(r["Counter_Name"], []).append(
                    (r["Kernel_Name"], int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return out


PER_PASS = [1]  # launches of one instantiation per pass (--launches-per-pass)


def mean(v):
    """per pass: the mean over launches of each kernel instantiation, summed
    over the instantiations (a chained pass of variant 0 launches its main and
    edge kernels, rb_tbc_kernel<..., 0> and <..., 1>, once each), times the
    launches per pass of one instantiation (the chained split ring runs its main
    and edge lists as two launches of the same rb_tbhc_kernel)"""
    by = {}
    for name, _, val in v:
        by.setdefault(name, []).append(val)
    return sum(sum(x) / len(x) for x in by.values()) * PER_PASS[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--iters", required=True,
                    help="iterations per pass of the launches to summarise, or 'all'")
    ap.add_argument("--kernel", default=None,
                    help="kernel name regex (default: the temporally blocked kernels, chained "
                         "rb_tbc_kernel or not, of ITERS iterations -- only full passes)")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--launches-per-pass", type=int, default=0,
                    help="launches of one instantiation per pass (0: 2 for rb_tbhc_kernel, "
                         "whose main and edge lists are two launches, else 1)")
    a = ap.parse_args()
    if a.iters == "all":
        ts = set()
        for path in glob.glob(os.path.join(a.dir, "**", "fetch*counter_collection.csv"),
                              recursive=True):
            for r in csv.DictReader(open(path)):
                m = re.search(r"rb_tb(?:hc|[cxh])?_kernel<(\d+),", r["Kernel_Name"])
                if m:
                    ts.add(int(m.group(1)))
        for t in sorted(ts):
            summarise(a, t, a.out.replace("{T}", str(t)))
    else:
        summarise(a, int(a.iters), a.out)


def summarise(a, iters, path_out):
    kernel = a.kernel or r"rb_tb(?:hc|[cxh])?_kernel<%d," % iters
    f = rows(a.dir, "fetch", kernel)
    PER_PASS[0] = a.launches_per_pass or (2 if any("rb_tbhc_kernel" in x[0] for v in f.values()
                                                   for x in v) else 1)
    w = rows(a.dir, "write", kernel)
    s = rows(a.dir, "sq", kernel)
    # full-iteration launches only (a capped solve's last pass may run fewer)
    fetch = f["FETCH_SIZE"]
    write = w["WRITE_SIZE"]
    rd = mean(fetch) * 1024 * 2
    wr = mean(write) * 1024
    cells = float(a.size) * a.size / a.nranks
    hbm_min = 24 * cells
    kname = fetch[0][0].split("(")[0].replace("void ", "")
    out = {
        "size": a.size, "nranks": a.nranks, "iters_per_pass": iters,
        "kernel": kname, "chain": bool(re.search(r"rb_tb(hc|c)_kernel", kname)),
        "rows_per_block": a.rows or None, "launches": len(fetch),
        "launches_per_pass": PER_PASS[0],
        "instantiations": sorted({x[0].split("(")[0].replace("void ", "") for x in fetch}),
        "fetch_size_kb_raw": mean(fetch), "write_size_kb": mean(write),
        "read_bytes_corrected": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
        "hbm_minimum_bytes_per_launch": hbm_min,
        "algorithmic_bytes_per_launch": hbm_min * iters,
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
            # lane-instructions per owned cell update (64 lanes per wave instruction)
            sq["valu_lane_insts_per_update"] = round(mean(s["SQ_INSTS_VALU"]) * 64 /
                                                     (cells * iters), 2)
        out["sq"] = sq
    out["note"] = ("one launch = %d solveRB iterations (temporally blocked); FETCH_SIZE x1024 x2 "
                   "(gfx950 correction, MI355X_MICROARCH.md HBM) + WRITE_SIZE x1024; separate "
                   "rocprofv3 --pmc passes (tools/profile_bench.sh); the HBM minimum of a launch "
                   "is 24 B x cells (p, rhs read once, p written once)" % iters)
    json.dump(out, open(path_out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
