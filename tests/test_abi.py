"""The C-ABI library loads on a GPU-less host and exports every entry point
include/misor.h declares; host-only entry points (decomposition) behave like
the reference's MPI topology code (assignment-5/skeleton/src/solver.c:30-32,
445-473)."""
import ctypes as C
import os
import re

import pytest

import pymisor as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "misor.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(misor3?_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = M.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    # and the binding covers exactly the declared ABI
    assert sorted(M.SIGNATURES) == syms


def test_version_string():
    assert b"gfx950" in M.lib().misor_version()


def mpi_dims_create(n):
    """MPI_Dims_create(n, 2): balanced, non-increasing"""
    best = max(d for d in range(1, int(n ** 0.5) + 1) if n % d == 0)
    return (n // best, best)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 6, 8, 12, 16])
def test_decompose_matches_mpi_topology(n):
    imax, jmax = 1001, 517
    dims = mpi_dims_create(n)
    covered = set()
    for r in range(n):
        loc = M.decompose(n, r, imax, jmax)
        assert tuple(loc.dims) == dims
        cx, cy = r // dims[1], r % dims[1]  # MPI_Cart_create row-major order
        assert tuple(loc.coords) == (cx, cy)
        # sizeOfRank: N/size + (N%size > rank)
        assert loc.ni == imax // dims[0] + (imax % dims[0] > cx)
        assert loc.nj == jmax // dims[1] + (jmax % dims[1] > cy)
        assert loc.ioff == sum(imax // dims[0] + (imax % dims[0] > c) for c in range(cx))
        assert loc.joff == sum(jmax // dims[1] + (jmax % dims[1] > c) for c in range(cy))
        nb = list(loc.neighbours)
        assert nb[0] == (r - dims[1] if cx > 0 else -1)
        assert nb[1] == (r + dims[1] if cx < dims[0] - 1 else -1)
        assert nb[2] == (r - 1 if cy > 0 else -1)
        assert nb[3] == (r + 1 if cy < dims[1] - 1 else -1)
        assert loc.pitch % 16 == 0 and loc.pitch >= loc.ni + 32
        covered.add((loc.ioff, loc.joff, loc.ni, loc.nj))
    assert sum(ni * nj for (_, _, ni, nj) in covered) == imax * jmax


def test_decompose_explicit_dims_and_errors():
    loc = M.decompose(8, 3, 64, 64, dims=(2, 4))
    assert tuple(loc.dims) == (2, 4)
    with pytest.raises(M.MisorError):
        M.decompose(8, 0, 64, 64, dims=(3, 3))
    with pytest.raises(M.MisorError):
        M.decompose(4, 4, 64, 64)
    M.decompose(64, 0, 64, 64)  # 8x8 ranks -> 8x8 cells each: fine
    with pytest.raises(M.MisorError):
        M.decompose(64, 63, 10, 10)  # 1x1 block on the last rank: rejected


def test_create_rejects_bad_descriptors():
    with pytest.raises(M.MisorError):
        M.Grid(1, 10, 1.0, 0.1, 1.9, 1e-6, 10)
    with pytest.raises(M.MisorError):
        M.Grid(10, 10, 0.0, 0.1, 1.9, 1e-6, 10)


def test_create3_rejects_bad_descriptors():
    prm = dict(imax=1, jmax=4, kmax=4, xlength=1.0, ylength=1.0, zlength=1.0, re=100.0,
               gamma=0.9, tau=0.5, omg=1.7, eps=1e-3, itermax=10, gx=0.0, gy=0.0, gz=0.0,
               bcTop=1, bcBottom=1, bcLeft=1, bcRight=1, bcFront=1, bcBack=1, name="dcavity")
    with pytest.raises(M.MisorError):
        M.Grid3(prm)


@pytest.mark.parametrize("n,kmax", [(1, 2), (2, 128), (3, 29), (8, 128), (8, 16)])
def test_decompose3_slabs(n, kmax):
    """slabs along k, sizeOfRank rule; every plane owned once"""
    off = 0
    for r in range(n):
        kl, ko = M.decompose3(n, r, kmax)
        assert ko == off and kl == kmax // n + (kmax % n > r) and kl >= 2
        off += kl
    assert off == kmax
    with pytest.raises(M.MisorError):
        M.decompose3(9, 0, 17)  # fewer than 2 planes per rank
    with pytest.raises(M.MisorError):
        M.decompose3(2, 2, 64)
