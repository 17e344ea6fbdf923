"""ctypes binding of libmisor (include/misor.h).

This is the Python-side stub of the C ABI: tests/, bench.py and
__graft_entry__.py drive the HIP path through it.  It loads the in-tree
lib/libmisor.so and fails loudly when that library is missing -- there is no
CPU fallback anywhere in the product path.

Host arrays are numpy float64 of shape (nj+2, ni+2): the reference layout
P(i,j) = p[j*(imax+2)+i] (assignment-4/src/solver.c:16) of this rank's block.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.path.join(HERE, "lib", "libmisor.so")
_DEFAULT_LIBPATH = LIBPATH

P, RHS, U, V, F, G = range(6)
NOSLIP, SLIP, OUTFLOW, PERIODIC = 1, 2, 3, 4
PROBLEM_NONE, PROBLEM_DCAVITY, PROBLEM_CANAL = 0, 1, 2
SOLVE_RB, SOLVE_RBA = 0, 1
LEX_A4, LEX_SEQ = 0, 1
(TUNE_SWEEP_VARIANT, TUNE_ROWS_PER_BLOCK, TUNE_XCD_REMAP, TUNE_SMALL_SOLVE, TUNE_OVERLAP,
 TUNE_TSTEPS, TUNE_TB_VARIANT, TUNE_TB_ROWS, TUNE_TB_PERSISTENT, TUNE_NS_FUSE,
 TUNE_FINISH2, TUNE_TB_RESERVE, TUNE_TB_CHAIN, TUNE_NEAR_BAND, TUNE_RES_LITE) = range(1, 16)
COMM_ID_BYTES = 128
# 3D field ids (misor3_*)
P3, RHS3, U3, V3, W3, F3, G3, H3 = range(8)
TUNE3_SWEEP, TUNE3_ROWS, TUNE3_KCHUNK, TUNE3_FOLD, TUNE3_RHS_AHEAD = 1, 2, 3, 4, 5
TUNE3_RESIDENT = 6  # whole solve in one cooperative launch, p in LDS (when it fits)

_dp = C.POINTER(C.c_double)


class Desc(C.Structure):
    _fields_ = [("imax", C.c_int), ("jmax", C.c_int), ("dx", C.c_double), ("dy", C.c_double),
                ("omega", C.c_double), ("eps", C.c_double), ("itermax", C.c_int),
                ("variant", C.c_int), ("device", C.c_int), ("nranks", C.c_int),
                ("rank", C.c_int), ("dims", C.c_int * 2), ("comm_id", C.c_void_p)]


class NsDesc(C.Structure):
    _fields_ = [("xlength", C.c_double), ("ylength", C.c_double), ("re", C.c_double),
                ("gx", C.c_double), ("gy", C.c_double), ("gamma", C.c_double),
                ("tau", C.c_double), ("bcLeft", C.c_int), ("bcRight", C.c_int),
                ("bcBottom", C.c_int), ("bcTop", C.c_int), ("problem", C.c_int)]


class Local(C.Structure):
    _fields_ = [("ni", C.c_int), ("nj", C.c_int), ("ioff", C.c_int), ("joff", C.c_int),
                ("coords", C.c_int * 2), ("dims", C.c_int * 2), ("neighbours", C.c_int * 4),
                ("pitch", C.c_longlong)]


class Stats(C.Structure):
    _fields_ = [("sweeps", C.c_longlong), ("launches", C.c_longlong), ("sweep_ms", C.c_double),
                ("timed_sweeps", C.c_longlong), ("timed_passes", C.c_longlong),
                ("iters_per_pass", C.c_int), ("tb_variant", C.c_int),
                ("halo_ms", C.c_double), ("halos", C.c_longlong),
                ("allreduce_ms", C.c_double), ("allreduces", C.c_longlong),
                ("chained", C.c_int), ("ns_ms", C.c_double * 3), ("ns_calls", C.c_longlong * 3),
                ("lite_misses", C.c_longlong)]


class Desc3(C.Structure):
    _fields_ = [("imax", C.c_int), ("jmax", C.c_int), ("kmax", C.c_int),
                ("xlength", C.c_double), ("ylength", C.c_double), ("zlength", C.c_double),
                ("re", C.c_double), ("gamma", C.c_double), ("tau", C.c_double),
                ("omega", C.c_double), ("eps", C.c_double),
                ("gx", C.c_double), ("gy", C.c_double), ("gz", C.c_double),
                ("itermax", C.c_int),
                ("bcTop", C.c_int), ("bcBottom", C.c_int), ("bcLeft", C.c_int),
                ("bcRight", C.c_int), ("bcFront", C.c_int), ("bcBack", C.c_int),
                ("problem", C.c_int), ("device", C.c_int), ("nranks", C.c_int),
                ("rank", C.c_int), ("comm_id", C.c_void_p)]


# every exported symbol of include/misor.h, with its ctypes signature
SIGNATURES = {
    "misor_last_error": (C.c_char_p, []),
    "misor_version": (C.c_char_p, []),
    "misor_decompose": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                  C.POINTER(Local)]),
    "misor_comm_unique_id": (C.c_int, [C.c_void_p]),
    "misor_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(Desc)]),
    "misor_destroy": (None, [C.c_void_p]),
    "misor_local_info": (C.c_int, [C.c_void_p, C.POINTER(Local)]),
    "misor_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "misor_synchronize": (C.c_int, [C.c_void_p]),
    "misor_upload": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "misor_download": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "misor_fill": (C.c_int, [C.c_void_p, C.c_int, C.c_double]),
    "misor_gather": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "misor_exchange": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "misor_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "misor_comm_ranks": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "misor_poisson_init": (C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_int]),
    "misor_solve_rb": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), _dp]),
    "misor_solve_rb_n": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int), _dp]),
    "misor_solve_lex": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int), _dp]),
    "misor_ns_setup": (C.c_int, [C.c_void_p, C.POINTER(NsDesc)]),
    "misor_compute_timestep": (C.c_int, [C.c_void_p, C.c_double, C.c_double, _dp]),
    "misor_set_dt": (C.c_int, [C.c_void_p, C.c_double]),
    "misor_set_boundary_conditions": (C.c_int, [C.c_void_p]),
    "misor_set_special_boundary_condition": (C.c_int, [C.c_void_p]),
    "misor_compute_fg": (C.c_int, [C.c_void_p]),
    "misor_compute_rhs": (C.c_int, [C.c_void_p]),
    "misor_normalize_pressure": (C.c_int, [C.c_void_p]),
    "misor_adapt_uv": (C.c_int, [C.c_void_p]),
    "misor_max_uv": (C.c_int, [C.c_void_p, _dp, _dp]),
    "misor_set_tuning": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "misor_get_tuning": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "misor_enable_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "misor_get_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "misor_reset_stats": (C.c_int, [C.c_void_p]),
    "misor_chain_trace": (C.c_int, [C.c_void_p, C.c_void_p, C.c_longlong,
                                    C.POINTER(C.c_longlong)]),
    "misor3_decompose": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int)]),
    "misor3_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(Desc3)]),
    "misor3_local_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "misor3_gather": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "misor3_destroy": (None, [C.c_void_p]),
    "misor3_upload": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "misor3_download": (C.c_int, [C.c_void_p, C.c_int, _dp]),
    "misor3_fill": (C.c_int, [C.c_void_p, C.c_int, C.c_double]),
    "misor3_set_dt": (C.c_int, [C.c_void_p, C.c_double]),
    "misor3_compute_timestep": (C.c_int, [C.c_void_p, _dp]),
    "misor3_max_uvw": (C.c_int, [C.c_void_p, _dp]),
    "misor3_set_boundary_conditions": (C.c_int, [C.c_void_p]),
    "misor3_set_special_boundary_condition": (C.c_int, [C.c_void_p]),
    "misor3_compute_fg": (C.c_int, [C.c_void_p]),
    "misor3_compute_rhs": (C.c_int, [C.c_void_p]),
    "misor3_solve": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), _dp]),
    "misor3_adapt_uvw": (C.c_int, [C.c_void_p]),
    "misor3_normalize_pressure": (C.c_int, [C.c_void_p]),
    "misor3_synchronize": (C.c_int, [C.c_void_p]),
    "misor3_enable_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "misor3_set_tuning": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "misor3_get_tuning": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "misor3_get_solve_time": (C.c_int, [C.c_void_p, _dp, C.POINTER(C.c_longlong)]),
}

_lib = None


class MisorError(RuntimeError):
    pass


# diagnostics that an older library (A/B runs) may lack; the default library must have all
_DIAGNOSTIC = {"misor_chain_trace"}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBPATH):
            raise MisorError("libmisor.so not built: run `make -C "
                             "practical-parallel-algorithms-with-mpi_amd` (or __graft_entry__.build())")
        L = C.CDLL(LIBPATH)
        for name, (res, args) in SIGNATURES.items():
            if name in _DIAGNOSTIC and LIBPATH != _DEFAULT_LIBPATH and not hasattr(L, name):
                continue  # an older library loaded for an A/B run (tools/scale_proxy.py --lib)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise MisorError("libmisor error %d: %s" % (rc, lib().misor_last_error().decode()))


def _ptr(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def decompose(nranks, rank, imax, jmax, dims=(0, 0)):
    loc = Local()
    d = (C.c_int * 2)(*dims)
    _check(lib().misor_decompose(nranks, rank, imax, jmax, d, C.byref(loc)))
    return loc


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib().misor_comm_unique_id(buf))
    return buf.raw


class Grid:
    """One rank's device-resident grid (the Solver struct's arrays in HBM)."""

    def __init__(self, imax, jmax, dx, dy, omega, eps, itermax, variant=SOLVE_RB, device=-1,
                 nranks=1, rank=0, dims=(0, 0), comm_id: bytes | None = None):
        d = Desc()
        d.imax, d.jmax, d.dx, d.dy = imax, jmax, dx, dy
        d.omega, d.eps, d.itermax, d.variant = omega, eps, itermax, variant
        d.device, d.nranks, d.rank = device, nranks, rank
        d.dims[0], d.dims[1] = dims
        self._id = C.create_string_buffer(comm_id, COMM_ID_BYTES) if comm_id else None
        d.comm_id = C.cast(self._id, C.c_void_p) if self._id is not None else None
        self.h = C.c_void_p()
        _check(lib().misor_create(C.byref(self.h), C.byref(d)))
        self.desc = d
        self.loc = Local()
        _check(lib().misor_local_info(self.h, C.byref(self.loc)))
        self.shape = (self.loc.nj + 2, self.loc.ni + 2)
        self.imax, self.jmax, self.rank, self.nranks = imax, jmax, rank, nranks

    def close(self):
        if self.h:
            lib().misor_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, field, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        assert a.shape == self.shape, (a.shape, self.shape)
        _check(lib().misor_upload(self.h, field, _ptr(a)))

    def download(self, field):
        a = np.empty(self.shape)
        _check(lib().misor_download(self.h, field, _ptr(a)))
        return a

    def gather(self, field):
        """collectResult: the global (jmax+2, imax+2) field on rank 0, None elsewhere
        (collective: every rank of the grid must call it)"""
        if self.rank == 0:
            out = np.empty((self.jmax + 2, self.imax + 2))
            _check(lib().misor_gather(self.h, field, _ptr(out)))
            return out
        _check(lib().misor_gather(self.h, field, C.cast(None, _dp)))
        return None

    def exchange(self, field, depth=1):
        """exchange (skeleton/src/solver.c:137-165): the depth-deep halo of
        `field` from the 8 neighbours (collective)"""
        _check(lib().misor_exchange(self.h, field, depth))

    def fill(self, field, value):
        _check(lib().misor_fill(self.h, field, value))

    def poisson_init(self, xlength, ylength, problem=2):
        _check(lib().misor_poisson_init(self.h, xlength, ylength, problem))

    def solve_rb(self, itermax=None):
        it = C.c_int(0)
        res = C.c_double(0.0)
        if itermax is None:
            _check(lib().misor_solve_rb(self.h, C.byref(it), C.byref(res)))
        else:
            _check(lib().misor_solve_rb_n(self.h, itermax, C.byref(it), C.byref(res)))
        return it.value, res.value

    def solve_lex(self, xorder=0):
        """lexicographic SOR (the reference's `solve`); xorder 0 = assignment-4,
        1 = assignment-5 sequential"""
        it, res = C.c_int(0), C.c_double(0.0)
        _check(lib().misor_solve_lex(self.h, xorder, C.byref(it), C.byref(res)))
        return it.value, res.value

    def synchronize(self):
        _check(lib().misor_synchronize(self.h))

    def comm_ranks(self):
        """ranks of the grid's communicator as the transport counts them
        (ncclCommCount for RCCL)"""
        n = C.c_int(0)
        _check(lib().misor_comm_ranks(self.h, C.byref(n)))
        return n.value

    def set_stream(self, stream_ptr):
        _check(lib().misor_set_stream(self.h, C.c_void_p(stream_ptr)))

    # ---- NS
    def ns_setup(self, prm: dict):
        n = NsDesc()
        n.xlength, n.ylength = prm["xlength"], prm["ylength"]
        n.re, n.gx, n.gy = prm["re"], prm["gx"], prm["gy"]
        n.gamma, n.tau = prm["gamma"], prm["tau"]
        n.bcLeft, n.bcRight = int(prm["bcLeft"]), int(prm["bcRight"])
        n.bcBottom, n.bcTop = int(prm["bcBottom"]), int(prm["bcTop"])
        n.problem = {"dcavity": PROBLEM_DCAVITY, "canal": PROBLEM_CANAL}.get(
            prm.get("name") or "", PROBLEM_NONE)
        _check(lib().misor_ns_setup(self.h, C.byref(n)))

    def compute_timestep(self, dt_bound, tau):
        dt = C.c_double(0.0)
        _check(lib().misor_compute_timestep(self.h, dt_bound, tau, C.byref(dt)))
        return dt.value

    def set_dt(self, dt):
        _check(lib().misor_set_dt(self.h, dt))

    def max_uv(self):
        a, b = C.c_double(0.0), C.c_double(0.0)
        _check(lib().misor_max_uv(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def call(self, name):
        _check(getattr(lib(), "misor_" + name)(self.h))

    # ---- tuning (launch geometry only; results are bit-identical)
    def set_tuning(self, key, value):
        _check(lib().misor_set_tuning(self.h, key, value))

    def get_tuning(self, key):
        v = C.c_int(0)
        _check(lib().misor_get_tuning(self.h, key, C.byref(v)))
        return v.value

    # ---- stats
    def enable_timing(self, on=True):
        _check(lib().misor_enable_timing(self.h, 1 if on else 0))

    def stats(self):
        s = Stats()
        _check(lib().misor_get_stats(self.h, C.byref(s)))
        return {"sweeps": s.sweeps, "launches": s.launches, "sweep_ms": s.sweep_ms,
                "timed_sweeps": s.timed_sweeps, "timed_passes": s.timed_passes,
                "iters_per_pass": s.iters_per_pass, "tb_variant": s.tb_variant,
                "halo_ms": s.halo_ms, "halos": s.halos,
                "allreduce_ms": s.allreduce_ms, "allreduces": s.allreduces,
                "chained": s.chained, "ns_ms": list(s.ns_ms), "ns_calls": list(s.ns_calls),
                "lite_misses": s.lite_misses}

    def reset_stats(self):
        _check(lib().misor_reset_stats(self.h))

    def chain_trace(self):
        """per-block timeline of the last chained pass (MISOR_CHAIN_TRACE=1 at
        configure time): array (blocks, 3) of start, end (100 MHz clock) and
        workgroup | 1 << 32 for a run's first block; None if not traced"""
        import numpy as np
        n = C.c_longlong(0)
        _check(lib().misor_chain_trace(self.h, None, 0, C.byref(n)))
        if n.value == 0:
            return None
        out = np.zeros(n.value, dtype=np.uint64)
        _check(lib().misor_chain_trace(self.h, out.ctypes.data, n.value, C.byref(n)))
        return out.reshape(-1, 3)


_PROBLEMS = {"dcavity": PROBLEM_DCAVITY, "canal": PROBLEM_CANAL}


def decompose3(nranks, rank, kmax):
    """(kloc, koff) of rank's slab"""
    a, b = C.c_int(0), C.c_int(0)
    _check(lib().misor3_decompose(nranks, rank, kmax, C.byref(a), C.byref(b)))
    return a.value, b.value


class Grid3:
    """The 3D solver (assignment-6/src/solver.c): fields of shape
    (kloc+2, jmax+2, imax+2), A(i,j,k) = a[k, j, i] (solver.c:19-34); kloc =
    kmax on one GPU, the rank's slab when decomposed (nranks > 1)."""

    def __init__(self, prm: dict, device=-1, nranks=1, rank=0, comm_id: bytes | None = None):
        d = Desc3()
        d.imax, d.jmax, d.kmax = int(prm["imax"]), int(prm["jmax"]), int(prm["kmax"])
        d.xlength, d.ylength, d.zlength = prm["xlength"], prm["ylength"], prm["zlength"]
        d.re, d.gamma, d.tau = prm["re"], prm["gamma"], prm["tau"]
        d.omega, d.eps, d.itermax = prm["omg"], prm["eps"], int(prm["itermax"])
        d.gx, d.gy, d.gz = prm["gx"], prm["gy"], prm["gz"]
        for k in ("bcTop", "bcBottom", "bcLeft", "bcRight", "bcFront", "bcBack"):
            setattr(d, k, int(prm[k]))
        d.problem = _PROBLEMS.get(prm.get("name") or "", PROBLEM_NONE)
        d.device = device
        d.nranks, d.rank = nranks, rank
        self._id = C.create_string_buffer(comm_id, COMM_ID_BYTES) if comm_id else None
        d.comm_id = C.cast(self._id, C.c_void_p) if self._id is not None else None
        self.h = C.c_void_p()
        _check(lib().misor3_create(C.byref(self.h), C.byref(d)))
        self.desc = d
        a, b = C.c_int(0), C.c_int(0)
        _check(lib().misor3_local_info(self.h, C.byref(a), C.byref(b)))
        self.kloc, self.koff = a.value, b.value
        self.rank, self.nranks = rank, nranks
        self.shape = (self.kloc + 2, d.jmax + 2, d.imax + 2)
        self.global_shape = (d.kmax + 2, d.jmax + 2, d.imax + 2)

    def close(self):
        if self.h:
            lib().misor3_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, field, arr):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        assert a.shape == self.shape, (a.shape, self.shape)
        _check(lib().misor3_upload(self.h, field, _ptr(a)))

    def download(self, field):
        a = np.empty(self.shape)
        _check(lib().misor3_download(self.h, field, _ptr(a)))
        return a

    def fill(self, field, value):
        _check(lib().misor3_fill(self.h, field, value))

    def gather(self, field):
        """the global field on rank 0, None elsewhere (collective)"""
        if self.rank == 0:
            out = np.empty(self.global_shape)
            _check(lib().misor3_gather(self.h, field, _ptr(out)))
            return out
        _check(lib().misor3_gather(self.h, field, C.cast(None, _dp)))
        return None

    def set_dt(self, dt):
        _check(lib().misor3_set_dt(self.h, dt))

    def compute_timestep(self):
        dt = C.c_double(0.0)
        _check(lib().misor3_compute_timestep(self.h, C.byref(dt)))
        return dt.value

    def max_uvw(self):
        m = (C.c_double * 3)()
        _check(lib().misor3_max_uvw(self.h, C.cast(m, _dp)))
        return tuple(m)

    def solve(self):
        it, res = C.c_int(0), C.c_double(0.0)
        _check(lib().misor3_solve(self.h, C.byref(it), C.byref(res)))
        return it.value, res.value

    def enable_timing(self, on=True):
        _check(lib().misor3_enable_timing(self.h, 1 if on else 0))

    def set_tuning(self, key, value):
        _check(lib().misor3_set_tuning(self.h, key, value))

    def get_tuning(self, key):
        v = C.c_int(0)
        _check(lib().misor3_get_tuning(self.h, key, C.byref(v)))
        return v.value

    def solve_time(self):
        """(device ms, iterations) of the solves timed since enable_timing"""
        ms, it = C.c_double(0.0), C.c_longlong(0)
        _check(lib().misor3_get_solve_time(self.h, C.byref(ms), C.byref(it)))
        return ms.value, it.value

    def call(self, name):
        """set_boundary_conditions, set_special_boundary_condition, compute_fg,
        compute_rhs, adapt_uvw, normalize_pressure, synchronize"""
        _check(getattr(lib(), "misor3_" + name)(self.h))
