#!/usr/bin/env python3
"""Interleaved A/B of the temporally blocked solve under different values of
one environment variable read by the library at launch (e.g. MISOR_TB_X of an
experiment build): each setting runs in its own child process per round (the
library reads the variable once), rounds interleaved; prints ms per iteration
(HIP events around every pass) and checks p is identical across settings.

    python tools/ab_env.py --lib lib_q/libmisor.so --var MISOR_TB_X --values 0,3,4 \
        --size 32768 --tsteps 7 --passes 6 --rounds 3
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
    import numpy as np
    import pymisor as M
    if a.lib:
        M.LIBPATH = os.path.abspath(a.lib)
    n, T = a.size, a.tsteps
    ni, nj = a.ni or n, a.nj or n
    g = M.Grid(ni, nj, 1.0 / n, 1.0 / n, 1.9, 1e-300, 1 << 20, device=0)
    if a.variant >= 0:
        g.set_tuning(M.TUNE_TB_VARIANT, a.variant)
    g.set_tuning(M.TUNE_TSTEPS, T)
    if a.rows:
        g.set_tuning(M.TUNE_TB_ROWS, a.rows)
    g.poisson_init(1.0, 1.0, 2)
    g.solve_rb(itermax=T)  # warm-up
    g.enable_timing(True)
    g.solve_rb(itermax=T * a.passes)  # (every instantiation of the plan has run)
    g.reset_stats()
    g.synchronize()
    import time
    t0 = time.perf_counter()
    g.solve_rb(itermax=T * a.passes)
    g.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / (T * a.passes)
    st = g.stats()
    p = g.download(M.P)
    h = float(np.sum(p[::97, ::89]))
    print(json.dumps({"ms_iter": st["sweep_ms"] / st["timed_sweeps"], "wall_iter": wall, "hash": h,
                      "rows": g.get_tuning(M.TUNE_TB_ROWS)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--var", default="MISOR_TB_X")
    ap.add_argument("--values", default="0")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--tsteps", type=int, default=7)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--ni", type=int, default=0, help="grid columns (default --size)")
    ap.add_argument("--nj", type=int, default=0, help="grid rows (default --size)")
    ap.add_argument("--variant", type=int, default=-1, help="TB variant (-1: default)")
    ap.add_argument("--passes", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    res = {}
    for r in range(a.rounds):
        for v in a.values.split(","):
            env = dict(os.environ, **{a.var: v})
            cmd = [sys.executable, __file__, "--child", "--size", str(a.size), "--tsteps",
                   str(a.tsteps), "--rows", str(a.rows), "--passes", str(a.passes),
                   "--ni", str(a.ni), "--nj", str(a.nj), "--variant", str(a.variant)]
            if a.lib:
                cmd += ["--lib", a.lib]
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit("child failed for %s=%s" % (a.var, v))
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
        print("round %d done" % r, file=sys.stderr, flush=True)
    hashes = {d["hash"] for v in res for d in res[v]}
    for v in res:
        ms = sorted(d["ms_iter"] for d in res[v])
        wl = sorted(d["wall_iter"] for d in res[v])
        print("%s=%s rows=%d ms/iter (events) med %.4f min %.4f | wall med %.4f min %.4f  "
              "MLUP/s (wall) %.0f" % (
                  a.var, v, res[v][0]["rows"], ms[len(ms) // 2], ms[0], wl[len(wl) // 2], wl[0],
                  float(a.ni or a.size) * (a.nj or a.size) / (wl[len(wl) // 2] * 1e-3) / 1e6))
    print("identical p across settings: %s" % (len(hashes) == 1))


if __name__ == "__main__":
    main()
