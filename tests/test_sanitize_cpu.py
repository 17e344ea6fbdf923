"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY 5:
the reference's failure mode is fail-fast; here memory errors, leaks and UB
in the CPU-side code are caught by a sanitized build).

Two executables, built by `make asan` (gcc -fsanitize=address,undefined
-fno-sanitize-recover=undefined):
  * bin/asan/host-check (practical-parallel-algorithms-with-mpi_amd/host/
    sanitize_main.c): the .par reader on every .par the tests use, the
    RCCL-id hand-off file (right tag taken, stale tag refused), the legacy
    VTK writer in both formats;
  * oracle/_asan/oracle-check (oracle/sanitize_main.c): every oracle
    function on small ragged grids, with the reference's iteration KATs and
    multi-threaded == scalar bit identity.
GPU code is not sanitized: GPU ASan / xnack+ runs are not available on this
pool, and the library's host-side C++ only runs inside the HIP library.
"""
import glob
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def build(d):
    subprocess.run(["make", "-s", "-C", d, "asan"], check=True, capture_output=True)


def run(cmd, **kw):
    r = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=300, **kw)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    return r.stdout


def test_host_code_sanitized(tmp_path):
    build(PKG)
    pars = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.par")))
    assert len(pars) >= 4
    out = run([os.path.join(PKG, "bin", "asan", "host-check"), str(tmp_path)] + pars)
    assert "all checks passed" in out
    assert (tmp_path / "sanitize_ascii.vtk").stat().st_size > 0


def test_oracle_sanitized():
    build(os.path.join(ROOT, "oracle"))
    out = run([os.path.join(ROOT, "oracle", "_asan", "oracle-check")])
    assert "all checks passed" in out
