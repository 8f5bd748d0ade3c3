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


def test_bench_skipped_collective_fails_fast():
    """One rank leaves out a collective: the others fail with the collective timeout (the
    init_process_group timeout, 5 s here), the launcher stops the job and exits non-zero with
    a message -- well inside its own wall-clock budget, never hanging."""
    import time
    t0 = time.monotonic()
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run",
              "--skip-collective-rank", "1", "--collective-timeout", "5",
              "--launch-timeout", "120"], timeout=150)
    took = time.monotonic() - t0
    assert p.returncode != 0, p.stdout
    assert took < 90, took
    assert "skipping a collective" in p.stderr
    assert "stopping the other ranks" in p.stderr or "budget" in p.stderr, p.stderr[-2000:]
    assert _json_lines(p.stdout) == []


def test_bench_launch_budget_stops_hung_ranks():
    """A rank that hangs past the launcher's wall-clock budget (collective timeout longer than
    the budget): the launcher SIGTERMs every rank and exits 124."""
    import time
    t0 = time.monotonic()
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run",
              "--skip-collective-rank", "1", "--collective-timeout", "600",
              "--launch-timeout", "15"], timeout=150)
    took = time.monotonic() - t0
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    assert took < 60, took
    assert "budget" in p.stderr


def test_bench_group_init_verifies_rank_ids():
    """The real run's group setup (init_group: timeout + a verified all-gather of the rank ids)
    is what --dry-run uses; its log line names the verified ids."""
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--dry-run"])
    assert p.returncode == 0, p.stderr
    assert "verified (rank-id all-gather [0, 1])" in p.stderr
