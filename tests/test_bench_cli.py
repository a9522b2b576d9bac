"""bench.py's launcher contract on the CPU (no GPU is touched on these paths):
* under a launcher, WORLD_SIZE must equal --gpus (else a non-zero exit before any work);
* --gpus N without a launcher spawns N child ranks with RANK / LOCAL_RANK / WORLD_SIZE set and
  exits non-zero when a rank fails (here cfg5, a single-GPU workload, refuses WORLD_SIZE=2 in
  each child before importing torch)."""
import os
import subprocess
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "does not match WORLD_SIZE=2" in r.stderr
    assert r.stdout == ""


def test_spawned_ranks_see_the_world_and_failures_propagate():
    r = _run(["--gpus", "2", "--workload", "cfg5"])
    assert r.returncode != 0
    # the children ran with WORLD_SIZE=2 and refused it (the parent stops the other rank once one
    # has failed, so it may not get to print)
    assert r.stderr.count("cfg5 is a single-GPU workload") >= 1, r.stderr
    assert r.stdout == ""
