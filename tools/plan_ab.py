#!/usr/bin/env python3
"""Pass-plan A/B on one rank's block: a capped solve of R iterations as the
library plans it by default, as T = 8 passes of the register-ring kernel
(variant 0, chained on blocks below 2^28 cells), and as T = 10 passes of the
chained split ring (variant 13), wall ms per iteration (median of rounds).

    python tools/plan_ab.py --shapes 32768x32768,16384x16384 --iters 20,100
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
    ap.add_argument("--shapes", default="32768x32768,16384x32768,16384x16384,8192x16384")
    ap.add_argument("--size", type=int, default=32768, help="spacing 1/size")
    ap.add_argument("--iters", default="20,100")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--comm", action="store_true", help="one-rank RCCL communicator (the "
                    "decomposed pipelined loop without neighbours)")
    a = ap.parse_args()
    iters = [int(x) for x in a.iters.split(",")]
    print("%-12s %5s %-10s %10s %8s %4s" % ("shape", "iters", "plan", "ms/iter", "T", "var"),
          flush=True)
    for sh in a.shapes.split(","):
        ni, nj = (int(x) for x in sh.split("x"))
        g = M.Grid(ni, nj, 1.0 / a.size, 1.0 / a.size, 1.9, 1e-300, max(iters), device=0,
                   comm_id=M.comm_unique_id() if a.comm else None)
        g.poisson_init(1.0, 1.0, 2)
        g.enable_timing(True)
        plans = {"default": (-1, -1), "t8": (0, 8), "hr10": (13, 10)}
        T0 = g.get_tuning(M.TUNE_TSTEPS)
        res = {}
        for rnd in range(a.rounds + 1):
            for name, (v, T) in plans.items():
                # (T first where it drops: variant 0 refuses T > 8)
                if v < 0:
                    g.set_tuning(M.TUNE_TSTEPS, T0)  # the default rule (no request)
                    g.set_tuning(M.TUNE_TB_VARIANT, 0)
                elif v == 0:
                    g.set_tuning(M.TUNE_TSTEPS, T)
                    g.set_tuning(M.TUNE_TB_VARIANT, v)
                else:
                    g.set_tuning(M.TUNE_TB_VARIANT, v)
                    g.set_tuning(M.TUNE_TSTEPS, T)
                for R in iters:
                    if rnd == 0:
                        g.solve_rb(itermax=R)
                        continue
                    g.reset_stats()
                    g.synchronize()
                    t0 = time.perf_counter()
                    g.solve_rb(itermax=R)
                    g.synchronize()
                    st = g.stats()
                    res.setdefault((name, R), []).append(
                        ((time.perf_counter() - t0) * 1e3 / R, st["iters_per_pass"],
                         st["tb_variant"]))
        for (name, R), v in sorted(res.items(), key=lambda x: (x[0][1], x[0][0])):
            print("%-12s %5d %-10s %10.4f %8d %4d" % (sh, R, name, np.median([x[0] for x in v]),
                                                      v[0][1], v[0][2]), flush=True)
        g.close()


if __name__ == "__main__":
    main()
