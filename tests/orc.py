"""ctypes access to the CPU oracle (oracle/liboracle.so) and, when it was built
in this container, to the reference itself (oracle/_ref/libref.so).

TEST INFRASTRUCTURE: only tests/, bench.py's cpu_baseline leg and
__graft_entry__.smoke() import this module.

Arrays are numpy float64 of shape (jmax+2, imax+2): row j, column i, exactly
the reference layout P(i,j) = p[j*(imax+2)+i] (assignment-4/src/solver.c:16).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIBORACLE = os.path.join(ORACLE_DIR, "liboracle.so")
LIBREF = os.path.join(ORACLE_DIR, "_ref", "libref.so")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)

NOSLIP, SLIP, OUTFLOW, PERIODIC = 1, 2, 3, 4
PROBLEM_NONE, PROBLEM_DCAVITY, PROBLEM_CANAL = 0, 1, 2


def _ptr(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def ensure_built():
    if not os.path.exists(LIBORACLE):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])


_lib = None


def lib():
    global _lib
    if _lib is None:
        ensure_built()
        L = C.CDLL(LIBORACLE)
        L.orc_poisson_init.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, _dp, _dp]
        for fn in (L.orc_solve_rb, L.orc_solve_rba):
            fn.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
                           C.c_int, _dp, _dp, _dp]
            fn.restype = C.c_int
        L.orc_solve_lex.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                    C.c_double, C.c_int, C.c_int, _dp, _dp, _dp]
        L.orc_solve_lex.restype = C.c_int
        L.orc_rb_pass_block.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_double, C.c_double, C.c_double, _dp, _dp]
        L.orc_rb_pass_block.restype = C.c_double
        L.orc_rb_pass_range.argtypes = [C.c_int] * 13 + [C.c_double] * 3 + [_dp, _dp]
        L.orc_rb_pass_range.restype = C.c_double
        for name in ("orc_ns_setup", "orc_ns_compute_timestep", "orc_ns_set_bc",
                     "orc_ns_set_special_bc", "orc_ns_compute_fg", "orc_ns_compute_rhs",
                     "orc_ns_normalize_pressure", "orc_ns_adapt_uv"):
            getattr(L, name).argtypes = [C.POINTER(OrcNS)]
        L.orc_ns_max_element.argtypes = [C.POINTER(OrcNS), _dp]
        L.orc_ns_max_element.restype = C.c_double
        L.orc_ns_run.argtypes = [C.POINTER(OrcNS), C.c_int, C.c_int, _ip, C.c_int, _dp]
        L.orc_ns_run.restype = C.c_int
        _lib = L
    return _lib


# ---------------------------------------------------------------- Poisson

def poisson_init(imax, jmax, xlength=1.0, ylength=1.0, problem=2):
    p = np.zeros((jmax + 2, imax + 2))
    rhs = np.zeros((jmax + 2, imax + 2))
    lib().orc_poisson_init(imax, jmax, xlength, ylength, problem, _ptr(p), _ptr(rhs))
    return p, rhs


def solve_rb(p, rhs, dx, dy, omega, eps, itermax, variant="rb"):
    """In place on p.  Returns (iterations, final res)."""
    jmax, imax = p.shape[0] - 2, p.shape[1] - 2
    res = C.c_double(0.0)
    fn = lib().orc_solve_rb if variant == "rb" else lib().orc_solve_rba
    it = fn(imax, jmax, dx, dy, omega, eps, itermax, _ptr(p), _ptr(rhs), C.byref(res))
    return it, res.value


def solve_rb_mt(p, rhs, dx, dy, omega, eps, itermax, nthreads):
    """multi-core solveRB (oracle_mt.c), in place on p"""
    L = lib()
    L.orc_solve_rb_mt.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                                  C.c_double, C.c_int, _dp, _dp, _dp, C.c_int]
    L.orc_solve_rb_mt.restype = C.c_int
    jmax, imax = p.shape[0] - 2, p.shape[1] - 2
    res = C.c_double(0.0)
    it = L.orc_solve_rb_mt(imax, jmax, dx, dy, omega, eps, itermax, _ptr(p), _ptr(rhs),
                           C.byref(res), nthreads)
    return it, res.value


def solve_lex(p, rhs, dx, dy, omega, eps, itermax, xorder=0):
    jmax, imax = p.shape[0] - 2, p.shape[1] - 2
    res = C.c_double(0.0)
    it = lib().orc_solve_lex(imax, jmax, dx, dy, omega, eps, itermax, xorder, _ptr(p),
                             _ptr(rhs), C.byref(res))
    return it, res.value


def rb_pass_block(p, rhs, ioff, joff, colour, idx2, idy2, factor):
    nj, ni = p.shape[0] - 2, p.shape[1] - 2
    return lib().orc_rb_pass_block(ni, nj, ioff, joff, colour, idx2, idy2, factor,
                                   _ptr(p), _ptr(rhs))


def sor_constants(dx, dy, omega):
    """The scalars solveRB derives (assignment-4/src/solver.c:185-189)."""
    dx2 = dx * dx
    dy2 = dy * dy
    return 1.0 / dx2, 1.0 / dy2, omega * 0.5 * (dx2 * dy2) / (dx2 + dy2)


# ---------------------------------------------------------------- NS

class OrcNS(C.Structure):
    _fields_ = [("imax", C.c_int), ("jmax", C.c_int), ("dx", C.c_double), ("dy", C.c_double),
                ("xlength", C.c_double), ("ylength", C.c_double), ("re", C.c_double),
                ("gx", C.c_double), ("gy", C.c_double), ("dt", C.c_double), ("te", C.c_double),
                ("tau", C.c_double), ("gamma", C.c_double), ("eps", C.c_double),
                ("omega", C.c_double), ("dtBound", C.c_double), ("itermax", C.c_int),
                ("bcLeft", C.c_int), ("bcRight", C.c_int), ("bcBottom", C.c_int),
                ("bcTop", C.c_int), ("problem", C.c_int),
                ("p", _dp), ("rhs", _dp), ("f", _dp), ("g", _dp), ("u", _dp), ("v", _dp)]


class NS:
    """Owns numpy fields and an OrcNS view of them (assignment-5/sequential
    initSolver semantics, solver.c:59-120)."""

    FIELDS = ("p", "rhs", "f", "g", "u", "v")

    def __init__(self, prm: dict):
        imax, jmax = int(prm["imax"]), int(prm["jmax"])
        shape = (jmax + 2, imax + 2)
        self.p = np.full(shape, float(prm.get("p_init", 0.0)))
        self.u = np.full(shape, float(prm.get("u_init", 0.0)))
        self.v = np.full(shape, float(prm.get("v_init", 0.0)))
        self.rhs = np.zeros(shape)
        self.f = np.zeros(shape)
        self.g = np.zeros(shape)
        s = OrcNS()
        s.imax, s.jmax = imax, jmax
        s.xlength, s.ylength = prm["xlength"], prm["ylength"]
        s.re, s.gx, s.gy = prm["re"], prm["gx"], prm["gy"]
        s.dt, s.te, s.tau, s.gamma = prm["dt"], prm["te"], prm["tau"], prm["gamma"]
        s.eps, s.omega, s.itermax = prm["eps"], prm["omg"], int(prm["itermax"])
        s.bcLeft, s.bcRight = int(prm["bcLeft"]), int(prm["bcRight"])
        s.bcBottom, s.bcTop = int(prm["bcBottom"]), int(prm["bcTop"])
        name = prm.get("name") or ""
        s.problem = {"dcavity": PROBLEM_DCAVITY, "canal": PROBLEM_CANAL}.get(name, PROBLEM_NONE)
        for k in self.FIELDS:
            setattr(s, k, _ptr(getattr(self, k)))
        self.s = s
        lib().orc_ns_setup(C.byref(s))

    def call(self, name):
        getattr(lib(), "orc_ns_" + name)(C.byref(self.s))

    def run(self, solver=1, max_steps=-1, cap=1 << 20):
        iters = np.zeros(cap, dtype=np.int32)
        t = C.c_double(0.0)
        n = lib().orc_ns_run(C.byref(self.s), solver, max_steps,
                             iters.ctypes.data_as(_ip), cap, C.byref(t))
        return n, iters[:min(n, cap)].copy(), t.value


def read_par(path):
    """Minimal Python reading of a .par for the oracle (key value # comment),
    with assignment-5/sequential/src/parameter.c:15-27 defaults."""
    prm = dict(xlength=1.0, ylength=1.0, imax=100, jmax=100, itermax=1000, eps=0.0001,
               omg=1.7, re=100.0, gamma=0.9, tau=0.5, gx=0.0, gy=0.0, dt=0.0, te=0.0,
               u_init=0.0, v_init=0.0, p_init=0.0, bcLeft=0, bcRight=0, bcBottom=0, bcTop=0,
               name=None)
    ints = {"imax", "jmax", "itermax", "bcLeft", "bcRight", "bcBottom", "bcTop"}
    with open(path) as fh:
        for line in fh:
            line = line.split("#", 1)[0].split()
            if len(line) < 2:
                continue
            k, v = line[0], line[1]
            if k in prm:
                prm[k] = v if k == "name" else (int(v) if k in ints else float(v))
    return prm


# ---------------------------------------------------------------- reference

_ref = None


def have_ref():
    return os.path.exists(LIBREF)


def ref():
    global _ref
    if _ref is None:
        R = C.CDLL(LIBREF)
        R.refa4_run.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, C.c_double,
                                C.c_double, C.c_int, C.c_int, _dp, _dp, _dp]
        R.refa4_run.restype = C.c_int
        R.refa4_write.argtypes = [C.c_int, C.c_int, _dp, C.c_char_p]
        R.refns_run.argtypes = [C.c_char_p, C.c_double, C.c_int, C.c_int, _ip, C.c_int, _dp,
                                _dp, _dp, _dp]
        R.refns_run.restype = C.c_int
        R.refa4_read_parameter.argtypes = [C.c_char_p, _ip, _ip, _ip, _dp, _dp, _dp, _dp]
        R.refa4_solve_rb_arrays.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double,
                                            C.c_double, C.c_double, C.c_int, _dp, _dp, _dp]
        R.refa4_solve_rb_arrays.restype = C.c_int
        R.refns_timed.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp,
                                  C.POINTER(C.c_longlong)]
        R.refns_timed.restype = C.c_int
        _ref = R
    return _ref


def ref_a4(imax, jmax, which="rb", itermax=1000000, eps=1e-6, omg=1.9, xlength=1.0,
           ylength=1.0, problem=2, init_p=None):
    p = np.zeros((jmax + 2, imax + 2))
    rhs = np.zeros((jmax + 2, imax + 2))
    w = {"lex": 0, "rb": 1, "rba": 2}[which]
    it = ref().refa4_run(imax, jmax, xlength, ylength, itermax, eps, omg, problem, w,
                         _ptr(init_p), _ptr(p), _ptr(rhs))
    return it, p, rhs


def ref_solve_rb_arrays(p, rhs, dx, dy, omega, eps, itermax):
    """the reference's solveRB in place on p (assignment-4/src/solver.c:179-238);
    returns (iterations, seconds of the solve alone)"""
    jmax, imax = p.shape[0] - 2, p.shape[1] - 2
    sec = C.c_double(0.0)
    it = ref().refa4_solve_rb_arrays(imax, jmax, dx, dy, omega, eps, itermax, _ptr(p),
                                     _ptr(rhs), C.byref(sec))
    return it, sec.value


def ref_ns_timed(par, imax, jmax, itermax, steps):
    """`steps` time steps of the reference's NS loop (composed with solveRB) on
    the .par's problem at imax x jmax, solve capped at itermax; returns
    (steps, seconds in solveRB, seconds of the steps, iterations)"""
    a, b, n = C.c_double(0.0), C.c_double(0.0), C.c_longlong(0)
    k = ref().refns_timed(par.encode(), imax, jmax, itermax, steps, C.byref(a), C.byref(b),
                          C.byref(n))
    return k, a.value, b.value, n.value


def ref_ns(par, te=-1.0, max_steps=-1, solver=1, cap=1 << 20):
    prm = read_par(par)
    shape = (prm["jmax"] + 2, prm["imax"] + 2)
    p, u, v = np.zeros(shape), np.zeros(shape), np.zeros(shape)
    iters = np.zeros(cap, dtype=np.int32)
    t = C.c_double(0.0)
    n = ref().refns_run(par.encode(), te, max_steps, solver, iters.ctypes.data_as(_ip), cap,
                        _ptr(p), _ptr(u), _ptr(v), C.byref(t))
    return n, iters[:min(n, cap)].copy(), p, u, v, t.value
