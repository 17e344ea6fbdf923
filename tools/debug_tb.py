#!/usr/bin/env python3
"""Where does the temporally blocked pass differ from the oracle?  Runs one
pass (itermax = T) on a grid with a forced block height and prints the error
pattern (rows, columns, strips, lanes, blocks) for several T / variants."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import orc  # noqa: E402
import pymisor as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ni", type=int, default=1700)
    ap.add_argument("--nj", type=int, default=900)
    ap.add_argument("--tsteps", default="2,3,5,7,9")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rows", default="0")
    ap.add_argument("--iters", default="T")
    ap.add_argument("--lib", default="")
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    if a.lib:
        M.LIBPATH = os.path.abspath(a.lib)
    ni, nj = a.ni, a.nj
    rng = np.random.default_rng(1)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    for T in map(int, a.tsteps.split(",")):
        k = T if a.iters == "T" else int(a.iters)
        want = p.copy()
        orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, k)
        for v in map(int, a.variants.split(",")):
            for rows in [int(r) for r in a.rows.split(",") for _ in range(a.reps)]:
                with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, k) as g:
                    g.set_tuning(M.TUNE_SMALL_SOLVE, 0)
                    g.set_tuning(M.TUNE_TSTEPS, T)
                    g.set_tuning(M.TUNE_TB_VARIANT, v)
                    g.set_tuning(M.TUNE_TB_ROWS, rows)
                    H = g.get_tuning(M.TUNE_TB_ROWS)
                    g.upload(M.P, p)
                    g.upload(M.RHS, rhs)
                    it, _ = g.solve_rb()
                    got = g.download(M.P)
                bad = np.argwhere(got != want)
                line = "T=%d v=%d rows=%d(H=%d) it=%d bad=%d" % (T, v, rows, H, it, len(bad))
                if len(bad):
                    ow = 128 - 4 * T
                    js, is_ = bad[:, 0], bad[:, 1]
                    strips = (is_ - 1) // ow
                    lanes = ((is_ - 1) % ow + 2 * T) // 2
                    line += " rows[%d..%d] uniq_rows=%d cols[%d..%d] strips=%s lanes=%s relrow=%s odd_cols=%.2f maxerr=%.3g" % (
                        js.min(), js.max(), len(set(js)), is_.min(), is_.max(),
                        sorted(set(strips.tolist()))[:12], sorted(set(lanes.tolist()))[:20],
                        sorted(set(((js - 1) % H).tolist()))[:20], (is_ % 2).mean(),
                        np.abs(got - want).max())
                print(line, flush=True)


if __name__ == "__main__":
    main()
