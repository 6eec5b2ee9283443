"""bench.py's rank layout on CPU: `python3 bench.py --gpus N` starts N ranks
by itself (torch.distributed.run as a child, nothing touches a GPU before), rank 0 alone prints
the one JSON line, and a WORLD_SIZE that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_2_self_launches_two_ranks_rank0_prints_once():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--dry-launch"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["dry_launch"] and out["n_gpus"] == 2 and out["comm"]["world_size"] == 2
    assert [q["rank"] for q in out["ranks"]] == [0, 1]
    assert sorted(q["local_rank"] for q in out["ranks"]) == [0, 1]
    assert len({q["pid"] for q in out["ranks"]}) == 2  # two processes, not one
    assert all(q["pid"] != os.getpid() for q in out["ranks"])


def test_world_size_disagreeing_with_gpus_is_refused():
    env = dict(_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-launch"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_1_runs_in_process_without_launcher():
    """--gpus 1 (the driver's N = 1 command) never starts a launcher: one rank, this process."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-launch"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert "launching" not in r.stderr
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1
