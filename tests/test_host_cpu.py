"""Host side of the drop-in (CPU): the .par reader of the host programs
(practical-parallel-algorithms-with-mpi_amd/host/parameter.c) against the
reference's own readParameter (assignment-4/src/parameter.c:26-67,
assignment-5/sequential/src/parameter.c:29-85) compiled into oracle/_ref,
on the reference's .par files and on edge cases of its line syntax."""
import ctypes as C
import os
import subprocess

import pytest

import orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAR_DUMP = os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd", "bin", "par-dump")

needs_ref = pytest.mark.skipif(not orc.have_ref(), reason="oracle/_ref not built")


class A5Parameter(C.Structure):  # assignment-5/sequential/src/parameter.h:10-21
    _fields_ = [("xlength", C.c_double), ("ylength", C.c_double), ("imax", C.c_int),
                ("jmax", C.c_int), ("itermax", C.c_int), ("eps", C.c_double),
                ("omg", C.c_double), ("re", C.c_double), ("tau", C.c_double),
                ("gamma", C.c_double), ("te", C.c_double), ("dt", C.c_double),
                ("gx", C.c_double), ("gy", C.c_double), ("name", C.c_char_p),
                ("bcLeft", C.c_int), ("bcRight", C.c_int), ("bcBottom", C.c_int),
                ("bcTop", C.c_int), ("u_init", C.c_double), ("v_init", C.c_double),
                ("p_init", C.c_double)]


def dump(path, poisson=False):
    out = subprocess.run([PAR_DUMP, path] + (["poisson"] if poisson else []),
                         capture_output=True, check=True).stdout.decode()  # keep \r
    lines = out.split("\n")
    d = {}
    k = 0
    while k < len(lines):
        line = lines[k]
        if line.startswith("name "):
            v = line[5:]
            if k + 1 < len(lines) and lines[k + 1] == "" and k + 2 < len(lines) and \
                    lines[k + 2].startswith("bcLeft"):
                v += "\n"  # the reference keeps a trailing newline in name
                k += 1
            d["name"] = v
        elif line:
            key, val = line.split(" ", 1)
            d[key] = val
        k += 1
    return d


def ref_a5(path):
    R = orc.ref()
    R.refns_read_parameter.argtypes = [C.c_char_p, C.POINTER(A5Parameter)]
    p = A5Parameter()
    R.refns_read_parameter(path.encode(), C.byref(p))
    return p


CASES = {
    "tabs_and_prefix.par": "xlength\t2.0\nylength 3.0 # c\nreynolds 42\nimax 17\t# x\n"
                           "jmax   9\nbcLeft 3\nbcTopx 2\nname canal\n"
                           "itermax 77\neps 1e-3\nomgX 1.1\n",
    "missing_values.par": "imax\njmax 12\n# only comment\n\nte 3.5\ndt\nu_init -1.25\n",
    "name_no_comment.par": "name dcavity\nimax 10\njmax 10\n",
    "last_line_no_newline.par": "imax 11\njmax 13",
}


@pytest.fixture(scope="module")
def par_files(tmp_path_factory, golden):
    d = tmp_path_factory.mktemp("par")
    files = [os.path.join(golden, f) for f in ("a6_dcavity.par", "a6_canal.par",
                                               "a4_poisson.par")]
    for name, txt in CASES.items():
        f = d / name
        f.write_text(txt)
        files.append(str(f))
    return files


@needs_ref
def test_reader_matches_reference_ns_reader(par_files):
    for path in par_files:
        mine = dump(path)
        ref = ref_a5(path)
        for name, ctype in A5Parameter._fields_:
            want = getattr(ref, name)
            got = mine[name]
            if name == "name":
                want = want.decode() if want is not None else "(null)"
                assert got == want, (path, name)
            elif ctype is C.c_int:
                assert int(got) == want, (path, name)
            else:
                assert float(got) == want, (path, name)


@needs_ref
def test_reader_matches_reference_poisson_reader(par_files):
    R = orc.ref()
    for path in par_files:
        mine = dump(path, poisson=True)
        v = [C.c_int(), C.c_int(), C.c_int(), C.c_double(), C.c_double(), C.c_double(),
             C.c_double()]
        R.refa4_read_parameter(path.encode(), *[C.byref(x) for x in v])
        imax, jmax, itermax, xl, yl, eps, omg = [x.value for x in v]
        assert (int(mine["imax"]), int(mine["jmax"]), int(mine["itermax"])) == \
            (imax, jmax, itermax), path
        assert (float(mine["xlength"]), float(mine["ylength"]), float(mine["eps"]),
                float(mine["omg"])) == (xl, yl, eps, omg), path


def test_reader_known_values(golden):
    d = dump(os.path.join(golden, "a6_canal.par"))
    assert d["name"] == "canal" and int(d["imax"]) == 200 and int(d["jmax"]) == 50
    assert float(d["xlength"]) == 30.0 and int(d["bcLeft"]) == 3 and int(d["itermax"]) == 500
    d = dump(os.path.join(golden, "a4_poisson.par"), poisson=True)
    assert float(d["omg"]) == 1.9 and int(d["itermax"]) == 1000000 and float(d["eps"]) == 1e-6


COMM_FILE = os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd", "bin", "comm-file")


@pytest.mark.parametrize("fetch_first", [True, False])
def test_comm_id_file_two_launches_in_a_row(tmp_path, fetch_first):
    """The RCCL id handshake of WORLD_SIZE > 1 launches (host/comm_file.c):
    two launches in a row with the same tag each hand their own id to the
    other ranks -- a reader never takes a file left by the previous launch
    (rank 0 removes it at the end and rewrites it atomically at the start),
    and a file of another launch tag is ignored"""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29511")
    env.pop("MISOR_COMM_FILE", None)
    env.pop("TORCHELASTIC_RUN_ID", None)
    env.pop("MISOR_RUN_TAG", None)
    # a stale file of ANOTHER launch at the same path must never be read
    stale = b"MISORID1" + b"other-launch".ljust(96, b"\0") + b"stale-id".ljust(128, b"\0")
    (tmp_path / "x.id").write_bytes(stale)
    env["MISOR_COMM_FILE"] = str(tmp_path / "x.id")
    for launch in ("first-id", "second-id"):
        readers = []
        if fetch_first:
            readers = [subprocess.Popen([COMM_FILE, "fetch", "3", str(k)], env=env,
                                        stdout=subprocess.PIPE) for k in (1, 2)]
        pub = subprocess.Popen([COMM_FILE, "publish", "3", launch, "2"], env=env)
        if not fetch_first:
            readers = [subprocess.Popen([COMM_FILE, "fetch", "3", str(k)], env=env,
                                        stdout=subprocess.PIPE) for k in (1, 2)]
        outs = [r.communicate(timeout=30)[0].decode().strip() for r in readers]
        assert pub.wait(timeout=30) == 0
        assert all(r.returncode == 0 for r in readers)
        assert outs == [launch, launch]
        assert not os.path.exists(env["MISOR_COMM_FILE"])
