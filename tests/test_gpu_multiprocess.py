"""GPU: the row-sharded path as real processes (`bench.py --gpus 2 --share-gpu`).

bench.py starts two ranks itself; both use GPU 0 and exchange the shared threshold, the
catalog-wide floor and the per-shard top-k over gloo (a one-GPU box cannot run two RCCL ranks).
Rank 0 then checks the merged global top-k of the last timed batch against the host float64
oracle over the whole catalog, regenerated from its seeds (bench.py:oracle_parity). This is the
multi-process protocol of the driver's N-GPU run -- rendezvous, async collectives, merge -- with
the parity check, at a catalog small enough for the suite (2 x 65536 rows x 1536, 512 queries).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


@pytest.mark.parametrize("world,n,b", [(2, 131072, 512), (8, 400_000, 1024)])
def test_bench_processes_share_gpu(cuda_device, world, n, b):
    """2 ranks on a small catalog; 8 ranks (the 8-GPU node's world size: shard_range and the
    shared sample tiles at world 8) on 50K-row shards. The N > 1 line carries the CPU baseline
    over the regenerated global catalog, the rescore stage time and a reason for the null
    traffic."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--share-gpu", "--config",
                        "C3", "--n", str(n), "--b", str(b), "--steps", "2", "--warmup", "1",
                        "--cpu-budget", "1", "--collective-timeout", "120",
                        "--launch-timeout", "280"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]            # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == world and "rehearsal" in j
    assert f"launched {world} ranks" in p.stderr
    assert f"rank-id all-gather {list(range(world))}" in p.stderr
    par = j["parity"]
    assert par["queries_checked"] >= 32
    assert par["rows_bit_exact"], par
    assert par["max_abs_score_diff"] <= 1e-12, par
    assert j["cpu_baseline"]["value"] > 0 and j["cpu_baseline"]["kind"] == "port"
    assert j["stage_ms_per_step"]["rescore"] > 0
    assert j["stage_ms_per_step"]["shard_merge"] > 0
    assert j["roofline"]["traffic"] is None and j["roofline"]["traffic_note"]
