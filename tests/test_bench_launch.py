"""bench.py --gpus G starts its G ranks itself: the parent launches one process
per GPU with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set before anything touches the GPU, so the
driver's plain `bench.py --gpus 8` runs config 4 on 8 ranks.  CPU only: the dry-run mode has every
rank report its environment and exit before any GPU work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("G", [2, 4, 8])
def test_launcher_starts_g_ranks(G):
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(G), "--launch-dry-run"], env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.strip()]
    assert sorted(x["rank"] for x in lines) == list(range(G))
    assert all(x["world"] == G and x["gpus"] == G and x["local_rank"] == x["rank"] for x in lines)
    assert all(x["master"] == "127.0.0.1" for x in lines)
    assert len({x["port"] for x in lines}) == 1


def test_world_size_mismatch_is_refused():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-dry-run"], env=env,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


def test_failing_rank_fails_the_launch():
    env = _env()
    env["ACCORD_DRY_FAIL_RANK"] = "1"
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-dry-run"], env=env,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 3
