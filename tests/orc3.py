"""ctypes access to the 3D CPU oracle (oracle/oracle3d.c, in liboracle.so)
and, when built in this container, to the reference's own 3D solver
(oracle/_ref/libref3d.so: assignment-6/src compiled in place).

TEST INFRASTRUCTURE ONLY.  Arrays are numpy float64 of shape
(kmax+2, jmax+2, imax+2): A(i,j,k) = a[k, j, i], the reference layout of
assignment-6/src/solver.c:19-34.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

import orc

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
LIBREF3 = os.path.join(orc.ORACLE_DIR, "_ref", "libref3d.so")
FIELDS = ("u", "v", "w", "p", "rhs", "f", "g", "h")


class Orc3(C.Structure):
    _fields_ = [("imax", C.c_int), ("jmax", C.c_int), ("kmax", C.c_int),
                ("xlength", C.c_double), ("ylength", C.c_double), ("zlength", C.c_double),
                ("dx", C.c_double), ("dy", C.c_double), ("dz", C.c_double),
                ("re", C.c_double), ("gx", C.c_double), ("gy", C.c_double),
                ("gz", C.c_double), ("dt", C.c_double), ("te", C.c_double),
                ("tau", C.c_double), ("gamma", C.c_double), ("eps", C.c_double),
                ("omega", C.c_double), ("dtBound", C.c_double), ("itermax", C.c_int),
                ("bcLeft", C.c_int), ("bcRight", C.c_int), ("bcBottom", C.c_int),
                ("bcTop", C.c_int), ("bcFront", C.c_int), ("bcBack", C.c_int),
                ("problem", C.c_int)] + [(n, _dp) for n in ("p", "rhs", "f", "g", "h", "u",
                                                            "v", "w")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = orc.lib()
        for n in ("orc3_setup", "orc3_compute_rhs", "orc3_normalize_pressure",
                  "orc3_compute_timestep", "orc3_set_bc", "orc3_set_special_bc",
                  "orc3_compute_fg", "orc3_adapt_uvw"):
            getattr(L, n).argtypes = [C.POINTER(Orc3)]
        L.orc3_solve.argtypes = [C.POINTER(Orc3), _dp]
        L.orc3_solve.restype = C.c_int
        L.orc3_max_element.argtypes = [C.POINTER(Orc3), _dp]
        L.orc3_max_element.restype = C.c_double
        L.orc3_run.argtypes = [C.POINTER(Orc3), C.c_int, _ip, C.c_int, _dp]
        L.orc3_run.restype = C.c_int
        L.orc3_collect.argtypes = [C.POINTER(Orc3), _dp, _dp, _dp, _dp]
        _lib = L
    return _lib


def read_par3(path):
    """assignment-6 .par (key value # comment) with the defaults of
    assignment-6/src/parameter.c:15-29 (keys it leaves unset: 0)"""
    prm = dict(xlength=1.0, ylength=1.0, zlength=1.0, imax=100, jmax=100, kmax=100,
               itermax=1000, eps=0.0001, omg=1.7, re=100.0, gamma=0.9, tau=0.5, gx=0.0,
               gy=0.0, gz=0.0, dt=0.0, te=0.0, u_init=0.0, v_init=0.0, w_init=0.0, p_init=0.0,
               bcLeft=0, bcRight=0, bcBottom=0, bcTop=0, bcFront=0, bcBack=0, name=None)
    ints = {"imax", "jmax", "kmax", "itermax", "bcLeft", "bcRight", "bcBottom", "bcTop",
            "bcFront", "bcBack"}
    with open(path) as fh:
        for line in fh:
            line = line.split("#", 1)[0].split()
            if len(line) < 2:
                continue
            k, v = line[0], line[1]
            if k in prm:
                prm[k] = v if k == "name" else (int(v) if k in ints else float(v))
    return prm


class NS3:
    """initSolver (assignment-6/src/solver.c:75-143) + the arrays"""

    def __init__(self, prm: dict):
        s = Orc3()
        for k in ("imax", "jmax", "kmax", "itermax", "bcLeft", "bcRight", "bcBottom", "bcTop",
                  "bcFront", "bcBack"):
            setattr(s, k, int(prm[k]))
        for k in ("xlength", "ylength", "zlength", "re", "gx", "gy", "gz", "dt", "te", "tau",
                  "gamma", "eps"):
            setattr(s, k, float(prm[k]))
        s.omega = float(prm["omg"])
        s.problem = {"dcavity": 1, "canal": 2}.get(prm.get("name") or "", 0)
        self.shape = (s.kmax + 2, s.jmax + 2, s.imax + 2)
        self.a = {n: np.zeros(self.shape) for n in FIELDS}
        self.a["u"][...] = prm.get("u_init", 0.0)
        self.a["v"][...] = prm.get("v_init", 0.0)
        self.a["w"][...] = prm.get("w_init", 0.0)
        self.a["p"][...] = prm.get("p_init", 0.0)
        for n in FIELDS:
            setattr(s, n, self.a[n].ctypes.data_as(_dp))
        self.s = s
        lib().orc3_setup(C.byref(s))

    def __getattr__(self, n):
        if n in FIELDS:
            return self.__dict__["a"][n]
        raise AttributeError(n)

    def call(self, name):
        getattr(lib(), "orc3_" + name)(C.byref(self.s))

    def solve(self):
        res = C.c_double(0.0)
        it = lib().orc3_solve(C.byref(self.s), C.byref(res))
        return it, res.value

    def run(self, max_steps=-1, cap=1 << 20):
        iters = np.zeros(cap, dtype=np.int32)
        t = C.c_double(0.0)
        n = lib().orc3_run(C.byref(self.s), max_steps, iters.ctypes.data_as(_ip), cap,
                           C.byref(t))
        return n, iters[:min(n, cap)].copy(), t.value

    def collect(self):
        n = self.s.imax * self.s.jmax * self.s.kmax
        out = [np.zeros(n) for _ in range(4)]
        lib().orc3_collect(C.byref(self.s), *[o.ctypes.data_as(_dp) for o in out])
        return out


# ------------------------------------------------------- the reference itself
_ref3 = None


def have_ref3():
    return os.path.exists(LIBREF3)


def ref3():
    global _ref3
    if _ref3 is None:
        R = C.CDLL(LIBREF3)
        R.ref3_run.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, _ip,
                               C.c_int, _dp, _dp, _dp, _dp, _dp]
        R.ref3_run.restype = C.c_int
        R.ref3_call.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp,
                                C.POINTER(_dp)]
        R.ref3_call.restype = C.c_int
        _ref3 = R
    return _ref3


REF_CALL = {"compute_timestep": 0, "set_bc": 1, "set_special_bc": 2, "compute_fg": 3,
            "compute_rhs": 4, "solve": 5, "adapt_uvw": 6, "normalize_pressure": 7}


def ref3_call(par, dims, which, dt, state):
    """run one reference function on `state` (dict of the 8 arrays, modified
    in place); returns (dt after, iterations for solve)"""
    arrs = [np.ascontiguousarray(state[n]) for n in FIELDS]
    ptrs = (_dp * 8)(*[a.ctypes.data_as(_dp) for a in arrs])
    d = C.c_double(dt)
    it = ref3().ref3_call(par.encode(), dims[0], dims[1], dims[2], REF_CALL[which],
                          C.byref(d), ptrs)
    for n, a in zip(FIELDS, arrs):
        state[n][...] = a
    return d.value, it


def ref3_run(par, dims=(0, 0, 0), te=-1.0, max_steps=-1, cap=1 << 20):
    prm = read_par3(par)
    imax, jmax, kmax = (dims[0] or prm["imax"], dims[1] or prm["jmax"], dims[2] or prm["kmax"])
    shape = (kmax + 2, jmax + 2, imax + 2)
    p, u, v, w = (np.zeros(shape) for _ in range(4))
    iters = np.zeros(cap, dtype=np.int32)
    t = C.c_double(0.0)
    n = ref3().ref3_run(par.encode(), dims[0], dims[1], dims[2], te, max_steps,
                        iters.ctypes.data_as(_ip), cap, *[a.ctypes.data_as(_dp)
                                                          for a in (p, u, v, w)], C.byref(t))
    return n, iters[:min(n, cap)].copy(), p, u, v, w, t.value
