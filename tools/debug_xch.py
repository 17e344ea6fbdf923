"""Diagnostics for the exchange TB kernel (variant 6): run small solves and
print where the field differs from the oracle (first rows / columns that
differ, per block row).  Usage: python tools/debug_xch.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import orc  # noqa: E402
import pymisor as M  # noqa: E402


def run(ni, nj, T, k, rows, variant=6, seed=1):
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 10
    dx, dy = 1.0 / ni, 1.3 / nj
    want = p.copy()
    orc.solve_rb(want, rhs, dx, dy, 1.8, 1e-300, k)
    with M.Grid(ni, nj, dx, dy, 1.8, 1e-300, k) as g:
        g.set_tuning(M.TUNE_SMALL_SOLVE, 0)
        g.set_tuning(M.TUNE_TB_VARIANT, variant)
        g.set_tuning(M.TUNE_TSTEPS, T)
        if rows:
            g.set_tuning(M.TUNE_TB_ROWS, rows)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        it, _ = g.solve_rb(itermax=k)
        got = g.download(M.P)
        st = g.stats()
    bad = got != want
    n = int(bad.sum())
    rows_bad = np.nonzero(bad.any(axis=1))[0]
    cols_bad = np.nonzero(bad.any(axis=0))[0]
    print("ni %d nj %d T %d k %d rows %d var %d: it %d passes %s bad %d  rows %s..%s  cols %s..%s"
          % (ni, nj, T, k, rows, variant, it, st["launches"], n,
             rows_bad[:1], rows_bad[-1:], cols_bad[:1], cols_bad[-1:]), flush=True)
    return n


if __name__ == "__main__":
    cases = [
        (615, 90, 4, 11, 12), (615, 90, 4, 4, 12), (615, 90, 4, 1, 12), (615, 90, 4, 2, 12),
        (615, 90, 4, 11, 24), (615, 190, 4, 11, 24), (1201, 90, 4, 11, 12),
        (615, 90, 8, 19, 28), (615, 90, 8, 8, 28), (1201, 700, 4, 4, 24), (1201, 700, 4, 4, 12),
        (616, 90, 4, 4, 12), (617, 90, 4, 4, 12), (400, 90, 4, 4, 12), (300, 190, 4, 4, 24),
    ]
    for c in cases:
        run(*c)
