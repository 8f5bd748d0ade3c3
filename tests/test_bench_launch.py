"""CPU: `bench.py --gpus N` starts and checks its own ranks (no external launcher needed).

The --dry-run mode runs the multi-rank protocol of a real run over gloo -- rendezvous on
127.0.0.1, the world-size check, barrier-bracketed steps, max-over-ranks timing and ONE JSON
line from rank 0 -- without the GPU path, so the launcher is covered here.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_gpus2_spawns_two_ranks():
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run"])
    assert p.returncode == 0, p.stderr
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout           # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and j["rccl_world_size"] == 2
    assert j["ranks_reported"] == [0, 1]        # both processes took part in the collective
    assert j["steps"] == 3 and j["warmup"] == 1
    assert "launched 2 ranks" in p.stderr


def test_bench_gpus1_unchanged():
    p = _run(["--gpus", "1", "--steps", "2", "--warmup", "0", "--dry-run"])
    assert p.returncode == 0, p.stderr
    (j,) = _json_lines(p.stdout)
    assert j["n_gpus"] == 1 and j["ranks_reported"] == [0]
    assert "launched" not in p.stderr


def test_bench_world_mismatch_fails():
    p = _run(["--gpus", "4", "--dry-run"], env_extra={"WORLD_SIZE": "2", "RANK": "0",
                                                      "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr
    assert _json_lines(p.stdout) == []
