"""A/B timing of the 3D solve variants (MISOR3_TUNE_*) on one GPU: fixed
iteration counts from a random state, device time from the library's HIP
events, p checked bit-identical across variants.

    python tools/tune3d.py --size 384 --iters 60 [--configs 1,8,0 1,4,0 0,8,0 ...]
    (a config is sweep,rows,kchunk[,fold[,rhs_ahead[,resident]]]; MISOR3_TUNE_*;
    resident defaults to 0 here)
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
import pymisor as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, nargs="+", default=[128, 384])
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default="", help="load this libmisor.so instead (A/B runs)")
    ap.add_argument("--configs", nargs="+",
                    default=["0,8,0", "1,4,0", "1,8,0", "1,12,0", "1,4,16", "1,8,16",
                             "1,8,64"])
    a = ap.parse_args()
    if a.lib:
        M.LIBPATH = os.path.abspath(a.lib)
    for n in a.size:
        prm = dict(imax=n, jmax=n, kmax=n, xlength=1.0, ylength=1.0, zlength=1.0, re=1000.0,
                   gamma=0.9, tau=0.5, omg=1.8, eps=1e-300, itermax=a.iters, gx=0.0, gy=0.0,
                   gz=0.0, bcTop=1, bcBottom=1, bcLeft=1, bcRight=1, bcFront=1, bcBack=1,
                   name="dcavity")
        rng = np.random.default_rng(1)
        p0 = rng.standard_normal((n + 2, n + 2, n + 2))
        rhs = rng.standard_normal((n + 2, n + 2, n + 2))
        ref = None
        for cfg in a.configs:
            v = [int(x) for x in cfg.split(",")]
            sw, rows, kc = v[:3]
            fold = v[3] if len(v) > 3 else 1
            ahead = v[4] if len(v) > 4 else 0
            res3 = v[5] if len(v) > 5 else 0
            with M.Grid3(prm) as g:
                g.set_tuning(M.TUNE3_SWEEP, sw)
                g.set_tuning(M.TUNE3_ROWS, rows)
                g.set_tuning(M.TUNE3_KCHUNK, kc)
                g.set_tuning(M.TUNE3_FOLD, fold)
                g.set_tuning(M.TUNE3_RHS_AHEAD, ahead)
                g.set_tuning(M.TUNE3_RESIDENT, res3)
                res3 = g.get_tuning(M.TUNE3_RESIDENT)
                g.upload(M.RHS3, rhs)
                best = None
                for r in range(a.reps + 1):
                    g.upload(M.P3, p0)
                    g.enable_timing(True)
                    it, _ = g.solve()
                    ms, its = g.solve_time()
                    if r > 0:
                        best = ms / its if best is None else min(best, ms / its)
                p = g.download(M.P3)
                same = "ref" if ref is None else ("same" if np.array_equal(p, ref) else "DIFF")
                if ref is None:
                    ref = p
                kc_eff = g.get_tuning(M.TUNE3_KCHUNK)
            mlups = n ** 3 / (best / 1e3) / 1e6
            print("n=%d sweep=%d rows=%d kc=%d fold=%d ahead=%d resident=%d: %.4f ms/iter  "
                  "%.0f MLUP/s  %.3f of 8 TB/s (24 B/LUP)  %s" % (
                      n, sw, rows, kc_eff, fold, ahead, res3, best, mlups, mlups * 24e-6 / 8.0,
                      same), flush=True)


if __name__ == "__main__":
    main()
