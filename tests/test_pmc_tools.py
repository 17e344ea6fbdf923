"""The PMC summary tools behind bench.py's `traffic` fields, on small
synthetic rocprofv3 counter files (CPU): the gfx950 correction (FETCH_SIZE KB x
1024 x 2 + WRITE_SIZE KB x 1024, MI355X_MICROARCH.md), one pass of the split
ring = two launches (main and edge lists), and the NS kernels' byte table."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]


def write_csv(path, rows):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(FIELDS, r)))


def run(tool, *args):
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", tool)] + list(args),
                          stdout=subprocess.DEVNULL)


def test_ns_summary_counts_two_launches_per_split_ring_pass(tmp_path):
    tb = "void misor::rb_tbhc_kernel<10, 4, 2, true, 1, 0, true>(misor::SweepParams)"
    fg = "void misor::fg_rhs_kernel<true>(misor::CLay)"
    d = tmp_path / "pmc"
    d.mkdir()
    # two passes: main launches 3000 / 2000 KB fetched, edge launches 1000 / 2000
    write_csv(d / "fetch_counter_collection.csv",
              [(1, tb, "FETCH_SIZE", 3000.0), (2, tb, "FETCH_SIZE", 1000.0),
               (3, tb, "FETCH_SIZE", 2000.0), (4, tb, "FETCH_SIZE", 2000.0),
               (5, fg, "FETCH_SIZE", 500.0)])
    write_csv(d / "write_counter_collection.csv",
              [(1, tb, "WRITE_SIZE", 800.0), (2, tb, "WRITE_SIZE", 200.0),
               (3, tb, "WRITE_SIZE", 600.0), (4, tb, "WRITE_SIZE", 400.0),
               (5, fg, "WRITE_SIZE", 300.0)])
    write_csv(d / "sq_counter_collection.csv",
              [(1, tb, "SQ_WAVE_CYCLES", 100.0), (1, tb, "SQ_ACTIVE_INST_VALU", 45.0)])
    out = tmp_path / "ns.json"
    run("ns_pmc_summary.py", str(d), str(out), "--size", "64")
    res = json.load(open(out))
    k = res["kernels"]["rb_tbhc_kernel"]
    # mean launch 2000 KB fetched x 2 launches per pass, x 1024 x 2 (gfx950)
    assert k["read_bytes_corrected"] == 2000.0 * 2 * 2048
    assert k["write_bytes"] == 500.0 * 2 * 1024
    assert k["algorithmic_bytes_per_launch"] == 24 * 64 * 64
    assert k["valu_busy_per_wave"] == 0.45
    f = res["kernels"]["fg_rhs_kernel"]
    assert f["bytes_per_launch"] == 500.0 * 2048 + 300.0 * 1024
    assert f["algorithmic_bytes_per_launch"] == 40 * 64 * 64
    assert res["solve_kernel"] == "rb_tbhc_kernel"


def test_pass_summary_of_the_bounded_split_ring(tmp_path):
    tb = "void misor::rb_tbhc_kernel<10, 4, 2, true, 1, 0, true>(misor::SweepParams)"
    d = tmp_path / "pmc"
    d.mkdir()
    write_csv(d / "fetch_counter_collection.csv",
              [(1, tb, "FETCH_SIZE", 4000.0), (2, tb, "FETCH_SIZE", 2000.0)])
    write_csv(d / "write_counter_collection.csv",
              [(1, tb, "WRITE_SIZE", 1000.0), (2, tb, "WRITE_SIZE", 1000.0)])
    out = tmp_path / "p.json"
    run("pmc_summary.py", str(d), str(out), "--size", "128", "--iters", "10")
    res = json.load(open(out))
    assert res["launches_per_pass"] == 2 and res["chain"]
    assert res["kernel"].startswith("misor::rb_tbhc_kernel<10")
    assert res["read_bytes_corrected"] == 3000.0 * 2 * 2048
    assert res["bytes_per_launch"] == 3000.0 * 2 * 2048 + 1000.0 * 2 * 1024
    assert res["hbm_minimum_bytes_per_launch"] == 24 * 128 * 128
