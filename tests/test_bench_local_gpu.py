"""bench.py's decomposed leg, run as in-process ranks on the one GPU of the
test box (--local-ranks: libmisor's LOCAL transport in place of RCCL, same
Grid code and pass loop): the N > 1 JSON line is produced -- comm block,
overlap -- and the gathered p after the timed solve equals a one-rank solve
of the same iterations bit for bit (SURVEY 8e partition independence).  What
the driver's 8-GPU SCALE run adds on top is RCCL itself."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n,size,scaling", [(2, 2048, "strong"), (4, 1536, "strong"),
                                            (8, 1024, "weak")])
def test_bench_local_ranks(n, size, scaling):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--local-ranks", str(n), "--size",
           str(size), "--steps", "20", "--warmup", "3", "--check", "--no-cpu-baseline",
           "--scaling", scaling]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["local_ranks"] == n and line["n_gpus"] == 1
    assert line["value"] > 0 and line["steps"] == 20
    c = line["comm"]
    assert c["halo_ms_per_exchange"] > 0 and c["sweep_ms_per_pass"] > 0
    assert c["overlap"] is None or 0.0 <= c["overlap"] <= 1.0
    assert line["check"]["p_bit_identical_to_1_rank"] is True
    dims = [int(x) for x in line["config"]["decomposition"].split("x")]
    assert dims[0] * dims[1] == n
