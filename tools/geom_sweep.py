#!/usr/bin/env python3
"""Block-geometry sweep of the temporally blocked pass on one rank's block (one
GPU, one process): for each local shape, every combination of block height
(MISOR_TB_TARGET_ROWS), short-block height (MISOR_TB_SMALL_ROWS) and band
rounds (MISOR_TB_BAND_ROUNDS) -- read by the library whenever it recomputes the
geometry -- in interleaved rounds; ms per iteration from the per-pass HIP events.

    python tools/geom_sweep.py --shapes 8192x16384 --tsteps 7 \
        --rows 153,187,221 --small 34,51 --band 1,2,3
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
    ap.add_argument("--shapes", default="8192x16384")
    ap.add_argument("--size", type=int, default=32768, help="global n (spacing 1/n)")
    ap.add_argument("--tsteps", type=int, default=7)
    ap.add_argument("--rows", default="0")
    ap.add_argument("--small", default="32")
    ap.add_argument("--band", default="2")
    ap.add_argument("--sweeps", type=int, default=56)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    combos = list(itertools.product(a.rows.split(","), a.small.split(","), a.band.split(",")))
    print("shape        T  rows small band  H_eff  ms/iter(med)  ms/iter(min)", flush=True)
    for sh in a.shapes.split(","):
        ni, nj = (int(x) for x in sh.split("x"))
        n = a.size
        g = M.Grid(ni, nj, 1.0 / n, 1.0 / n, 1.9, 1e-300, a.sweeps, device=0)
        g.poisson_init(ni / n, nj / n, 2)
        g.enable_timing(True)
        res = {c: [] for c in combos}
        heff = {}
        for rnd in range(a.rounds + 1):
            for c in combos:
                os.environ["MISOR_TB_TARGET_ROWS"], os.environ["MISOR_TB_SMALL_ROWS"], \
                    os.environ["MISOR_TB_BAND_ROUNDS"] = c
                g.set_tuning(M.TUNE_TSTEPS, a.tsteps)  # recompute the geometry
                heff[c] = g.get_tuning(M.TUNE_TB_ROWS)
                g.reset_stats()
                g.solve_rb(itermax=a.sweeps)
                st = g.stats()
                if rnd > 0:  # the first round warms every geometry up
                    res[c].append(st["sweep_ms"] / max(st["timed_sweeps"], 1))
        for c in combos:
            print("%-12s %2d %4s %5s %4s  %5d  %12.4f  %12.4f" % (
                sh, a.tsteps, c[0], c[1], c[2], heff[c], float(np.median(res[c])),
                float(np.min(res[c]))), flush=True)
        g.close()


if __name__ == "__main__":
    main()
