#!/usr/bin/env python3
"""A/B the sweep kernel's launch variants in ONE process, interleaved
(cdna_hip_programming.md §5.4 rule 24), at a given grid size.

    python tools/tune_sweep.py [--size 32768] [--sweeps 10] [--rounds 3]

Prints one line per (variant, rows_per_block, xcd_remap) with the median and
min sweep-kernel time (HIP events around each launch) and the algorithmic
GB/s (24 B per lattice update).  Also checks that every setting produces the
same bits as the first one.

    python tools/tune_sweep.py --tb --tsteps 1,2,3,4 --variants 0,1,2,3 --rows 64,128,256

tunes the multi-iteration (temporally blocked) kernel instead: per-iteration
time = pass time / T, GB/s = 24 B x cells x T / pass time (algorithmic).
"""
import argparse
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
import pymisor as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--sweeps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--rows", default="0,64,256")
    ap.add_argument("--remap", default="0,1")
    ap.add_argument("--tb", action="store_true")
    ap.add_argument("--tsteps", default="2,3,4")
    ap.add_argument("--lib", default="", help="load this libmisor.so instead (A/B builds)")
    args = ap.parse_args()
    if args.lib:
        M.LIBPATH = os.path.abspath(args.lib)
    if args.tb:
        return main_tb(args)
    n = args.size
    g = M.Grid(n, n, 1.0 / n, 1.0 / n, 1.9, 1e-300, args.sweeps, device=0)
    g.poisson_init(1.0, 1.0, 2)
    g.enable_timing(True)
    combos = list(itertools.product([int(v) for v in args.variants.split(",")],
                                    [int(r) for r in args.rows.split(",")],
                                    [int(x) for x in args.remap.split(",")]))
    times = {c: [] for c in combos}
    for rnd in range(args.rounds):
        for c in combos:
            v, rows, remap = c
            g.set_tuning(M.TUNE_SWEEP_VARIANT, v)
            g.set_tuning(M.TUNE_ROWS_PER_BLOCK, rows)
            g.set_tuning(M.TUNE_XCD_REMAP, remap)
            g.reset_stats()
            g.solve_rb(itermax=args.sweeps)
            st = g.stats()
            times[c].append(st["sweep_ms"] / st["timed_sweeps"])
        print("round %d done" % rnd, file=sys.stderr, flush=True)
    # bit-identity across settings (fresh field each, 3 sweeps)
    ref = None
    small = 4099
    h = M.Grid(small, 1031, 1.0 / small, 1.0 / 1031, 1.9, 1e-300, 3, device=0)
    for c in combos:
        v, rows, remap = c
        h.set_tuning(M.TUNE_SWEEP_VARIANT, v)
        h.set_tuning(M.TUNE_ROWS_PER_BLOCK, rows)
        h.set_tuning(M.TUNE_XCD_REMAP, remap)
        h.poisson_init(1.0, 1.0, 2)
        h.solve_rb()
        p = h.download(M.P)
        if ref is None:
            ref = p
        assert np.array_equal(p, ref), c
    cells = float(n) * n
    print("%-8s %5s %5s %10s %10s %8s" % ("variant", "rows", "remap", "med_ms", "min_ms", "GB/s"))
    for c in sorted(combos, key=lambda c: np.median(times[c])):
        med, mn = np.median(times[c]), np.min(times[c])
        print("%-8d %5d %5d %10.4f %10.4f %8.1f" % (c[0], c[1], c[2], med, mn,
                                                   24.0 * cells / (med * 1e-3) / 1e9))
    print("bit-identical across settings: yes")


def main_tb(args):
    n = args.size
    sweeps = args.sweeps
    g = M.Grid(n, n, 1.0 / n, 1.0 / n, 1.9, 1e-300, sweeps, device=0)
    g.poisson_init(1.0, 1.0, 2)
    g.enable_timing(True)
    combos = list(itertools.product([int(t) for t in args.tsteps.split(",")],
                                    [int(v) for v in args.variants.split(",")],
                                    [int(r) for r in args.rows.split(",")]))
    times = {c: [] for c in combos}
    for rnd in range(args.rounds):
        # untimed lead-in: the first solve of a round runs slow (clocks ramp)
        g.set_tuning(M.TUNE_TSTEPS, combos[0][0])
        g.solve_rb(itermax=combos[0][0] * max(1, args.sweeps // combos[0][0]))
        for c in combos:
            T, v, rows = c
            g.set_tuning(M.TUNE_TSTEPS, T)
            g.set_tuning(M.TUNE_TB_VARIANT, v)
            g.set_tuning(M.TUNE_TB_ROWS, rows)
            g.reset_stats()
            g.solve_rb(itermax=T * max(1, args.sweeps // T))  # whole passes of T
            st = g.stats()
            assert st["iters_per_pass"] == T
            times[c].append(st["sweep_ms"] / st["timed_sweeps"])  # per iteration
        print("round %d done" % rnd, file=sys.stderr, flush=True)
    ref = None
    small = 4099
    h = M.Grid(small, 1031, 1.0 / small, 1.0 / 1031, 1.9, 1e-300, 7, device=0)
    h.set_tuning(M.TUNE_SMALL_SOLVE, 0)
    for c in combos:
        T, v, rows = c
        h.set_tuning(M.TUNE_TSTEPS, T)
        h.set_tuning(M.TUNE_TB_VARIANT, v)
        h.set_tuning(M.TUNE_TB_ROWS, rows)
        h.poisson_init(1.0, 1.0, 2)
        h.solve_rb()
        p = h.download(M.P)
        if ref is None:
            ref = p
        assert np.array_equal(p, ref), c
    cells = float(n) * n
    print("%-3s %-8s %5s %12s %12s %8s" % ("T", "variant", "rows", "med_ms/iter",
                                           "min_ms/iter", "GB/s"))
    for c in sorted(combos, key=lambda c: np.median(times[c])):
        med, mn = np.median(times[c]), np.min(times[c])
        print("%-3d %-8d %5d %12.4f %12.4f %8.1f" % (c[0], c[1], c[2], med, mn,
                                                     24.0 * cells / (med * 1e-3) / 1e9))
    print("bit-identical across settings: yes")


if __name__ == "__main__":
    main()
