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


def test_bench_two_processes_share_gpu(cuda_device):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--share-gpu", "--config", "C3",
                        "--n", "131072", "--b", "512", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]            # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and "rehearsal" in j
    assert "launched 2 ranks" in p.stderr
    par = j["parity"]
    assert par["queries_checked"] == 32
    assert par["rows_bit_exact"], par
    assert par["max_abs_score_diff"] <= 1e-12, par
