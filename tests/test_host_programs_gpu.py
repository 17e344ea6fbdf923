"""The reference-compatible host programs (C, on libmisor) end to end:
bin/exe-poisson <par> like assignment-4/src/main.c, bin/exe-ns <par> like
assignment-5/sequential/src/main.c -- stdout lines, output files, results."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd", "bin")


def fmt_pdat(p):  # writeResult, assignment-4/src/solver.c:315-320
    return "\n".join("".join("%f " % x for x in row) for row in p) + "\n"


def test_exe_poisson(golden, tmp_path):
    shutil.copy(os.path.join(golden, "a4_poisson.par"), tmp_path / "poisson.par")
    out = subprocess.run([os.path.join(BIN, "exe-poisson"), "poisson.par"], cwd=tmp_path,
                         capture_output=True, text=True, timeout=120, check=True).stdout
    assert "Parameters:" in out and "Cells (x, y): 100, 100" in out
    assert re.search(r"(^|\s)2388 ", out), out
    assert re.search(r"Walltime \d+\.\d\ds", out)
    z = np.load(os.path.join(golden, "rb_poisson100.npz"))
    assert (tmp_path / "p.dat").read_text() == fmt_pdat(z["p"])


def test_exe_ns_dcavity(golden, tmp_path):
    z = np.load(os.path.join(golden, "ns_dcavity_rb_short.npz"))
    txt = open(os.path.join(golden, "a6_dcavity.par")).read()
    txt = re.sub(r"(?m)^te .*$", "te       %r" % float(z["te"]), txt)
    (tmp_path / "dcavity.par").write_text(txt)
    env = dict(os.environ, MISOR_ITERLOG=str(tmp_path / "iters.log"))
    out = subprocess.run([os.path.join(BIN, "exe-ns"), "dcavity.par"], cwd=tmp_path, env=env,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    assert "Parameters for dcavity" in out and "Solution took" in out
    log = np.loadtxt(tmp_path / "iters.log")
    assert len(log) == int(z["steps"])
    assert np.array_equal(log[:, 3].astype(int), z["iters"])
    # pressure.dat: "%.2f %.2f %f" per interior cell, blank line after each row
    pr = np.loadtxt(tmp_path / "pressure.dat")
    assert pr.shape == (128 * 128, 3)
    assert np.abs(pr[:, 2] - z["p"][1:-1, 1:-1].ravel()).max() <= 1e-6
    ve = np.loadtxt(tmp_path / "velocity.dat")
    u, v = z["u"], z["v"]
    uc = ((u[1:-1, 1:-1] + u[1:-1, :-2]) / 2.0).ravel()
    vc = ((v[1:-1, 1:-1] + v[:-2, 1:-1]) / 2.0).ravel()
    assert np.abs(ve[:, 2] - uc).max() <= 1e-6
    assert np.abs(ve[:, 3] - vc).max() <= 1e-6


@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_exe_poisson_decomposed(golden, tmp_path, ranks):
    """MISOR_RANKS=N: N ranks (threads, in-process transport) on a 2D
    decomposition, p assembled on rank 0 (collectResult) -> the same p.dat"""
    shutil.copy(os.path.join(golden, "a4_poisson.par"), tmp_path / "poisson.par")
    env = dict(os.environ, MISOR_RANKS=str(ranks))
    out = subprocess.run([os.path.join(BIN, "exe-poisson"), "poisson.par"], cwd=tmp_path,
                         env=env, capture_output=True, text=True, timeout=120, check=True).stdout
    assert out.count("Parameters:") == 1 and out.count("Walltime") == 1
    assert re.search(r"(^|\s)2388 ", out), out
    z = np.load(os.path.join(golden, "rb_poisson100.npz"))
    assert (tmp_path / "p.dat").read_text() == fmt_pdat(z["p"])


@pytest.mark.parametrize("par,ranks", [("a6_dcavity.par", 4), ("a6_canal.par", 2),
                                       ("a6_canal.par", 4)])
def test_exe_ns_decomposed_matches_single(golden, tmp_path, par, ranks):
    """the NS program decomposed over N ranks writes the same pressure.dat /
    velocity.dat as on one GPU and takes the same pressure iterations per step"""
    name = par[3:]
    txt = open(os.path.join(golden, par)).read()
    # (dcavity on 4 in-process ranks: ~0.2 s a step on its small grid -- the
    # transport's per-pass host barriers -- so a shorter run)
    te = 0.15 if (par, ranks) == ("a6_dcavity.par", 4) else 0.3
    txt = re.sub(r"(?m)^te .*$", "te       %r" % te, txt)
    runs = {}
    for n in (1, ranks):
        d = tmp_path / ("r%d" % n)
        d.mkdir()
        (d / name).write_text(txt)
        env = dict(os.environ, MISOR_RANKS=str(n), MISOR_ITERLOG=str(d / "iters.log"))
        out = subprocess.run([os.path.join(BIN, "exe-ns"), name], cwd=d, env=env,
                             capture_output=True, text=True, timeout=300, check=True).stdout
        assert out.count("Solution took") == 1
        runs[n] = d
    a, b = runs[1], runs[ranks]
    la, lb = np.loadtxt(a / "iters.log"), np.loadtxt(b / "iters.log")
    assert la.shape == lb.shape and len(la) > 3
    assert np.array_equal(la[:, 3], lb[:, 3])  # pressure iterations per step
    # dt is a max-reduction (order-free) and normalizePressure's sum is exact,
    # so every field and every dt is bit-identical for any partition
    assert np.array_equal(la[:, 2], lb[:, 2])
    for f in ("pressure.dat", "velocity.dat"):
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


def test_exe_poisson_lexicographic_reproduces_committed_pdat(golden, tmp_path):
    """MISOR_SOLVER=lex: the reference's own solve (assignment-4/src/main.c:34
    calls the lexicographic SOR) -> its committed p.dat, byte for byte"""
    shutil.copy(os.path.join(golden, "a4_poisson.par"), tmp_path / "poisson.par")
    env = dict(os.environ, MISOR_SOLVER="lex")
    out = subprocess.run([os.path.join(BIN, "exe-poisson"), "poisson.par"], cwd=tmp_path,
                         env=env, capture_output=True, text=True, timeout=120, check=True).stdout
    assert re.search(r"(^|\s)2388 ", out), out
    assert (tmp_path / "p.dat").read_text() == open(os.path.join(golden, "a4_p.dat")).read()


def test_exe_ns_lexicographic_short(golden, tmp_path):
    """MISOR_SOLVER=lex: the reference's sequential NS on its dcavity.par
    (100 steps; the 400-step run is test_lex_gpu.py's) -> pressure.dat /
    velocity.dat of the reference build's fields"""
    z = np.load(os.path.join(golden, "ns_seq_dcavity_lex_100.npz"))
    txt = open(os.path.join(golden, "seq_dcavity.par")).read()
    txt = re.sub(r"(?m)^te .*$", "te       %r" % float(z["te"]), txt)
    (tmp_path / "dcavity.par").write_text(txt)
    env = dict(os.environ, MISOR_SOLVER="lex", MISOR_ITERLOG=str(tmp_path / "iters.log"))
    subprocess.run([os.path.join(BIN, "exe-ns"), "dcavity.par"], cwd=tmp_path, env=env,
                   capture_output=True, text=True, timeout=300, check=True)
    assert len(np.loadtxt(tmp_path / "iters.log")) == int(z["steps"])
    pr = np.loadtxt(tmp_path / "pressure.dat")
    assert np.abs(pr[:, 2] - z["p"][1:-1, 1:-1].ravel()).max() <= 1e-6
    ve = np.loadtxt(tmp_path / "velocity.dat")
    u, v = z["u"], z["v"]
    assert np.abs(ve[:, 2] - ((u[1:-1, 1:-1] + u[1:-1, :-2]) / 2.0).ravel()).max() <= 1e-6
    assert np.abs(ve[:, 3] - ((v[1:-1, 1:-1] + v[:-2, 1:-1]) / 2.0).ravel()).max() <= 1e-6
