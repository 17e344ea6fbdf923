#!/usr/bin/env python3
"""HBM bytes per launch of the NS config-5 kernels (bench.py --workload ns)
from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu/run.sh
ns), with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE KB x 1024 x
2 + WRITE_SIZE KB x 1024), against each kernel's algorithmic bytes per cell:
fg_rhs 40 (u, v in; f, g, rhs out), adapt_absmax 40 (f, g, p in; u, v out),
the solve's pass 24 (p, rhs in; p out), and normalizePressure's three
kernels -- absmax2 8 (p in), exact_sum 8 (p in), sub_mean 16 (p in and out) --
also summed as "normalize_pressure" (32).

    python tools/ns_pmc_summary.py gpurun_out/TAG/ns_pmc profiles/r06_pmc_ns16384.json --size 16384
"""
import argparse
import collections
import csv
import glob
import json
import os

# kernel name fragment -> algorithmic bytes per cell
KERNELS = {"fg_rhs_kernel": 40, "adapt_absmax_kernel": 40, "rb_tb_kernel": 24,
           "rb_tbc_kernel": 24, "rb_tbhc_kernel": 24, "absmax2_kernel": 8,
           "exact_sum_kernel": 8, "sub_mean_kernel": 16}
NORMALIZE = ("absmax2_kernel", "exact_sum_kernel", "sub_mean_kernel")


def per_kernel(d, prefix, counter):
    acc = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", prefix + "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            for k in KERNELS:
                if "::%s<" % k in name or "::%s(" % k in name or name.startswith(k):
                    acc[k].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--nranks", type=int, default=1)
    a = ap.parse_args()
    fetch = per_kernel(a.dir, "fetch", "FETCH_SIZE")
    write = per_kernel(a.dir, "write", "WRITE_SIZE")
    cyc = per_kernel(a.dir, "sq", "SQ_WAVE_CYCLES")
    vbusy = per_kernel(a.dir, "sq", "SQ_ACTIVE_INST_VALU")
    cells = a.size * a.size
    res = {"size": a.size, "nranks": a.nranks, "kernels": {}}
    for k in sorted(fetch):
        if k not in write:
            continue
        # the split ring runs a pass as two launches (main and edge lists):
        # bytes per pass = the mean launch x 2
        per = 2 if k == "rb_tbhc_kernel" else 1
        f = sum(fetch[k]) / len(fetch[k]) * per
        w = sum(write[k]) / len(write[k]) * per
        b = f * 1024 * 2 + w * 1024
        alg = KERNELS[k] * cells
        res["kernels"][k] = {"launches": len(fetch[k]), "fetch_size_kb_raw": f,
                             "write_size_kb": w, "read_bytes_corrected": f * 2048,
                             "write_bytes": w * 1024, "bytes_per_launch": b,
                             "algorithmic_bytes_per_launch": alg,
                             "ratio_to_algorithmic": b / alg}
        if cyc.get(k) and vbusy.get(k):
            res["kernels"][k]["valu_busy_per_wave"] = round(sum(vbusy[k]) / sum(cyc[k]), 3)
    if all(k in res["kernels"] for k in NORMALIZE):
        b = sum(res["kernels"][k]["bytes_per_launch"] for k in NORMALIZE)
        res["kernels"]["normalize_pressure"] = {
            "bytes_per_launch": b, "algorithmic_bytes_per_launch": 32 * cells,
            "ratio_to_algorithmic": b / (32 * cells), "parts": list(NORMALIZE)}
    solve = [k for k in ("rb_tbhc_kernel", "rb_tbc_kernel", "rb_tb_kernel") if k in res["kernels"]]
    if solve:
        res["solve_kernel"] = solve[0]
    res["note"] = ("separate rocprofv3 --pmc passes of bench.py --workload ns; FETCH_SIZE x1024 x2 "
                   "(gfx950: 128-B requests tallied at 64 B) + WRITE_SIZE x1024; the solve kernel's "
                   "bytes are per pass (rb_tbhc_kernel: two launches per pass, main and edge "
                   "lists); valu_busy_per_wave = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main()
