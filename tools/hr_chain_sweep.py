#!/usr/bin/env python3
"""A/B of the chained split-ring pass geometry (sor_tbh.h rb_tbhc_kernel):
block height in ring lengths (MISOR_TB_CHAIN_RINGS) and the cost the segment
plan gives a block of a column at a physical left / right side
(MISOR_CHAIN_EDGE_COST), against the unchained pass, on one rank's block.

    python tools/hr_chain_sweep.py --shape 32768x32768 --rings 4,8,16 --edge 2,3.4
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
import pymisor as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="32768x32768")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--T", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rings", default="4,8,16")
    ap.add_argument("--edge", default="2,3.4")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    ni, nj = (int(x) for x in a.shape.split("x"))
    g = M.Grid(ni, nj, 1.0 / a.size, 1.0 / a.size, 1.9, 1e-300, a.iters, device=0)
    g.poisson_init(1.0, 1.0, 2)
    g.set_tuning(M.TUNE_TB_VARIANT, 13)
    g.set_tuning(M.TUNE_TSTEPS, a.T)
    g.enable_timing(True)
    combos = [(0, 0, 0.0)] + [(1, int(r), float(e)) for r in a.rings.split(",")
                              for e in a.edge.split(",")]
    res = {c: [] for c in combos}
    for rnd in range(a.rounds + 1):
        for c in combos:
            ch, r, e = c
            os.environ["MISOR_TB_CHAIN_RINGS"] = str(r or 4)
            os.environ["MISOR_CHAIN_EDGE_COST"] = str(e or 2.0)
            g.set_tuning(M.TUNE_TB_CHAIN, ch)  # rebuilds the geometry and plans
            g.solve_rb(itermax=a.T)  # plan build, first launch
            g.reset_stats()
            g.synchronize()
            t0 = time.perf_counter()
            it, _ = g.solve_rb(itermax=a.iters)
            g.synchronize()
            wall = (time.perf_counter() - t0) * 1e3 / a.iters
            st = g.stats()
            if rnd:
                res[c].append((wall, st["sweep_ms"] / max(st["timed_passes"], 1),
                               g.get_tuning(M.TUNE_TB_ROWS)))
    print("%-10s %5s %5s %5s %10s %10s" % ("shape", "chain", "rows", "edge", "ms/iter", "ms/pass"))
    for c in combos:
        ch, r, e = c
        w = np.median([x[0] for x in res[c]])
        p = np.median([x[1] for x in res[c]])
        print("%-10s %5d %5d %5.1f %10.4f %10.3f" % (a.shape, ch, res[c][0][2], e, w, p), flush=True)
    g.close()


if __name__ == "__main__":
    main()
