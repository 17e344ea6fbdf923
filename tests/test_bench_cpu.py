"""bench.py's process plumbing on the CPU (no GPU call): --gpus N > 1 without a
launcher spawns N workers with the environment torch.distributed.run would
give them; a WORLD_SIZE that disagrees with --gpus is an error; --dry-run
stops every worker before its first GPU call."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
LAUNCH_VARS = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
               "MASTER_PORT", "GROUP_RANK")


def _run(args, extra_env=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_spawn_assigns_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # one JSON line, from the spawning parent
    d = json.loads(lines[0])
    assert d["dry_run"] and d["spawned"] == n and d["exit_codes"] == [0] * n
    ws = sorted(d["workers"], key=lambda w: w["rank"])
    assert [w["rank"] for w in ws] == list(range(n))
    assert [w["local_rank"] for w in ws] == list(range(n))
    assert all(w["world_size"] == n and w["gpus"] == n for w in ws)
    assert all(w["device"] == "cuda:%d" % w["local_rank"] for w in ws)
    assert {w["master_addr"] for w in ws} == {"127.0.0.1"}
    assert {w["master_port"] for w in ws} == {str(d["master_port"])}


def test_one_gpu_needs_no_launcher():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert (d["rank"], d["local_rank"], d["world_size"]) == (0, 0, 1)


def test_launcher_env_is_used():
    # under torch.distributed.run: the launcher's variables, no spawning
    r = _run(["--gpus", "4", "--dry-run"],
             {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3", "MASTER_ADDR": "127.0.0.1",
              "MASTER_PORT": "29512"})
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert (d["rank"], d["local_rank"], d["world_size"], d["master_port"]) == (3, 3, 4, "29512")


@pytest.mark.parametrize("world,gpus", [("2", "4"), ("8", "1"), ("1", "8")])
def test_world_size_mismatch_fails(world, gpus):
    r = _run(["--gpus", gpus, "--dry-run"], {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr and not r.stdout.strip()
