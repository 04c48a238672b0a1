"""bench.py's multi-GPU launcher (the driver runs ``bench.py --gpus N``): N > 1
without WORLD_SIZE starts N rank processes itself, as the reference's mp.spawn
does (MSFNO/main.py:1149-1156).  ``--dry-run`` stops after the process group
(gloo) is up, so this runs on the CPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240, cwd=REPO)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == d["world_size"] == d["ranks_seen"] == n
    if n > 1:
        assert len(d["pids"]) == n and os.getpid() not in d["pids"]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_failed_rank_fails_the_job():
    # an unknown filter is rejected by argparse in every rank: the launcher returns non-zero
    r = _run(["--gpus", "2", "--dry-run", "--filter", "nope"])
    assert r.returncode != 0
