"""CPU: bench.py's multi-rank launcher and max-over-ranks aggregation (gloo self-test mode).

`python bench.py --gpus N` without WORLD_SIZE starts N ranks through a child
`torch.distributed.run` (never an exec of a process that touched the GPU); rank 0 prints one
JSON line.  The --selftest-cpu step is a tiny CPU matmul, so this covers exactly the launch,
rendezvous (127.0.0.1), barrier and reduction plumbing the GPU run uses.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2])
def test_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--selftest-cpu", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["world_size"] == n and d["steps"] == 3
    assert d["backend"] == ("gloo" if n > 1 else None)


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--selftest-cpu"], env_extra={"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
