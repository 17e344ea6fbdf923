#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

Every vector below is produced by oracle/_ref/libref.so, i.e. the reference's
own C sources (assignment-4/src/solver.c, assignment-5/sequential/src/*.c)
compiled in place by oracle/Makefile (-O2 -ffp-contract=off).  The GPU box has
no /root/reference, so the tests read these committed .npz files instead.

Fixtures:
  rb_kat.json              solveRB iteration counts, poisson.par family
  rb_poisson100.npz        solveRB on assignment-4/poisson.par: p, iterations
  rb_sweeps.npz            p after 1/2/7 solveRB sweeps on odd/ragged grids
  ns_dcavity_rb_short.npz  composed RB-NS, a6 dcavity.par, te=0.5
  ns_canal_rb_short.npz    composed RB-NS, a6 canal.par, te=2
  ns_dcavity_rb_full.npz   composed RB-NS, a6 dcavity.par, te=10 (per-step iters + fields)
  ns3d_dcavity_short.npz / ns3d_canal_short.npz  the reference's 3D NS (assignment-6/src,
                           oracle/_ref/libref3d.so) on its dcavity/canal .par at reduced
                           grids, 16 time steps: per-step iterations, p, u, v, w, t
  ns_seq_dcavity_lex_100.npz    the same run to te=0.0125 (100 steps): p, u, v, t
  ns_seq_dcavity_lex_short.npz  the reference's own NS (assignment-5/sequential, its
                           lexicographic `solve`) on its dcavity.par, te=0.05: p, u, v,
                           t, and the per-step iteration counts of the restatement
                           (iters_oracle: the shipped solve() reports none)
plus reference data files copied verbatim (they are the reference's own
fixtures): a4_p.dat, a4_init.dat, and assignment-5/sequential's dcavity.par,
pressure.dat and velocity.dat (seq_*; the committed output of its te=10 run).
"""
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import orc  # noqa: E402

REF = "/root/reference"
A6 = os.path.join(REF, "assignment-6")


SEQ = os.path.join(REF, "assignment-5/sequential")


def lex_fixtures():
    """the reference's lexicographic NS (its actual `solve`)"""
    for name in ("dcavity.par", "pressure.dat", "velocity.dat"):
        shutil.copyfile(os.path.join(SEQ, name), os.path.join(HERE, "seq_" + name))
    te = 0.05
    n, _, p, u, v, t = orc.ref_ns(os.path.join(SEQ, "dcavity.par"), te=te, solver=0)
    # per-step iteration counts: the reference's shipped solve() reports none
    # (oracle/ref_glue.c), so they come from the restatement -- whose fields
    # are checked against these reference fields bit for bit (test_oracle.py)
    prm = orc.read_par(os.path.join(SEQ, "dcavity.par"))
    prm["te"] = te
    ns = orc.NS(prm)
    n_o, iters_o, _ = ns.run(solver=0)
    assert n_o == n and np.array_equal(ns.p, p) and np.array_equal(ns.u, u)
    np.savez_compressed(os.path.join(HERE, "ns_seq_dcavity_lex_short.npz"), steps=n,
                        iters_oracle=np.asarray(iters_o, dtype=np.int32), p=p, u=u, v=v, t=t,
                        te=te)
    print("ns_seq_dcavity_lex_short.npz", n, "steps")
    # a shorter run of the same (te = 0.0125, 100 steps) for the host-program test
    te = 0.0125
    n, _, p, u, v, t = orc.ref_ns(os.path.join(SEQ, "dcavity.par"), te=te, solver=0)
    np.savez_compressed(os.path.join(HERE, "ns_seq_dcavity_lex_100.npz"), steps=n, p=p, u=u,
                        v=v, t=t, te=te)
    print("ns_seq_dcavity_lex_100.npz", n, "steps")


def ns3d_fixtures():
    """the reference's 3D NS (assignment-6/src/main.c loop) at reduced grids"""
    import orc3
    assert orc3.have_ref3(), "build oracle/_ref first: make -C oracle ref"
    for par, dims, out in (("dcavity.par", (24, 20, 16), "ns3d_dcavity_short.npz"),
                           ("canal.par", (40, 12, 10), "ns3d_canal_short.npz")):
        n, iters, p, u, v, w, t = orc3.ref3_run(os.path.join(A6, par), dims=dims,
                                                max_steps=16)
        np.savez_compressed(os.path.join(HERE, out), steps=n, iters=iters, p=p, u=u, v=v,
                            w=w, t=t, dims=np.array(dims))
        print(out, n, "steps", int(iters.sum()), "iterations")


def main(full=True):
    assert orc.have_ref(), "build oracle/_ref first: make -C oracle ref"
    lex_fixtures()
    ns3d_fixtures()

    # reference data fixtures
    shutil.copyfile(os.path.join(REF, "assignment-4/p.dat"), os.path.join(HERE, "a4_p.dat"))
    shutil.copyfile(os.path.join(REF, "assignment-4/init.dat"), os.path.join(HERE, "a4_init.dat"))
    for name in ("dcavity.par", "canal.par"):
        shutil.copyfile(os.path.join(A6, name), os.path.join(HERE, "a6_" + name))
    shutil.copyfile(os.path.join(REF, "assignment-4/poisson.par"), os.path.join(HERE, "a4_poisson.par"))

    # 1. iteration-count KATs (poisson.par family: omega 1.9, eps 1e-6, problem 2)
    kat = {}
    for n in (50, 64, 100, 128, 200):
        it, _, _ = orc.ref_a4(n, n, "rb")
        kat[str(n)] = it
    for (ni, nj) in ((64, 32), (33, 75)):
        it, _, _ = orc.ref_a4(ni, nj, "rb")
        kat["%dx%d" % (ni, nj)] = it
    with open(os.path.join(HERE, "rb_kat.json"), "w") as fh:
        json.dump({"omega": 1.9, "eps": 1e-6, "problem": 2, "xlength": 1.0, "ylength": 1.0,
                   "iterations": kat}, fh, indent=1)

    # 2. poisson.par to convergence
    it, p, _ = orc.ref_a4(100, 100, "rb")
    itl, pl, _ = orc.ref_a4(100, 100, "lex")
    np.savez_compressed(os.path.join(HERE, "rb_poisson100.npz"), p=p, iterations=it,
                        p_lex=pl, iterations_lex=itl)

    # 3. fixed sweep counts on ragged grids (itermax = k, eps tiny)
    cases = {}
    for (ni, nj, xl, yl) in ((5, 3, 1.0, 1.0), (37, 23, 1.0, 2.0), (130, 17, 3.0, 1.0),
                             (129, 64, 1.0, 1.0), (256, 9, 2.0, 0.5)):
        for k in (1, 2, 7):
            it, p, _ = orc.ref_a4(ni, nj, "rb", itermax=k, eps=1e-300, xlength=xl, ylength=yl)
            assert it == k
            cases["p_%dx%d_k%d" % (ni, nj, k)] = p
        cases["geom_%dx%d" % (ni, nj)] = np.array([ni, nj, xl, yl])
    np.savez_compressed(os.path.join(HERE, "rb_sweeps.npz"), **cases)

    # 4. composed red-black NS (assignment-5/sequential + assignment-4 solveRB)
    def ns(par, te, out):
        n, iters, p, u, v, t = orc.ref_ns(os.path.join(A6, par), te=te, solver=1)
        np.savez_compressed(os.path.join(HERE, out), steps=n, iters=iters, p=p, u=u, v=v,
                            t=t, te=te)
        print(out, n, "steps", int(iters.sum()), "sweeps")

    ns("dcavity.par", 0.5, "ns_dcavity_rb_short.npz")
    ns("canal.par", 2.0, "ns_canal_rb_short.npz")
    if full:
        ns("dcavity.par", 10.0, "ns_dcavity_rb_full.npz")


if __name__ == "__main__":
    if "--lex-only" in sys.argv:
        lex_fixtures()
    elif "--3d-only" in sys.argv:
        ns3d_fixtures()
    else:
        main(full="--short" not in sys.argv)
