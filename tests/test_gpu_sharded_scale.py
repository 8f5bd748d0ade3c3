"""GPU: the row-sharded protocol at the 8-GPU configurations' real shapes, before the driver's
first 8-GPU run.

Eight ranks are simulated by eight threads on one MI355X (tests/test_gpu_sharded.py:
ThreadCollectives -- the same tensors, in the same order, as all_gather_into_tensor), each rank
holding its shard_range block of the bench's own seeded catalog (bench.make_catalog_shard) with
global row ids through row_offset, and driving bench.py's N > 1 loop
(distributed.run_sharded_steps over score_topk_sharded_local_stages: two batches in flight,
the catalog-wide floor, per-shard retries). Checked per configuration:
  * every rank returns the same merged answer;
  * it equals the single-GPU path over the whole catalog bit for bit (rows and scores);
  * sampled queries equal the host float64 oracle (oracle.restatement.cosine_topk_stream, the
    catalog streamed to the host in row blocks): rows bit-exact, |ds| <= 1e-12;
  * properties of every query: scores non-increasing, rows unique and in range, no excluded row.
Shapes (BASELINE.json configs):
  C3/8  1M x 1536 f32, 4096 queries, top-100, 125K rows per shard: the SHARED screening
        threshold branch (shared_sample_tiles > 0), with 128 excluded rows per query;
  C4/8  the whole 10M x 768 bf16 catalog (15.4 GB, one GPU holds it), 8192 queries, top-100:
        1.25M rows per shard, per-shard speculative screens + the floor cut;
  C5/8  8 x 1M x 1536 f16 (the C5 batch and k on 1M-row shards instead of 6.25M), 16384
        queries, top-1000: k' = 1256 > 512, the floor-only branch with block merges.
Reference: /root/reference/src/backend/app/lib.py:51-55 (what every shard restates).
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import restatement as R
from test_gpu_sharded import _run_sharded
from test_gpu_workloads import device_blocks

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WORLD = 8
SCORE_ATOL = 1e-12


def _queries(cfg, seed, dev):
    import bench
    c = dict(cfg)
    g = torch.Generator(device=dev).manual_seed(seed)
    q = torch.randn((c["b"], c["d"]), generator=g, device=dev, dtype=torch.float32)
    return q.to(bench.TORCH_DT[c["dtype"]])


def _check_properties(s, r, n, excl=None):
    sn, rn = s.cpu().numpy(), r.cpu().numpy()
    assert np.all(np.isfinite(sn)) and np.all(rn >= 0) and np.all(rn < n)
    assert np.all(np.diff(sn, axis=1) <= 0)
    assert np.all(np.abs(sn) <= 1 + 1e-12)
    assert np.all(np.diff(np.sort(rn, axis=1), axis=1) > 0), "duplicate rows in a top-k"
    if excl is not None:
        for b in range(0, rn.shape[0], 13):
            assert not np.isin(rn[b], excl[b]).any()


def _log(msg):
    import time
    print(f"[scale {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _sharded_at_scale(cuda_device, cfg, n_sample, excl_per_query=0, check_plan=None,
                      path="python", slots=2):
    import bench
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import (ShardedTopk, TorchGatherComm, run_sharded_steps,
                                             score_topk_sharded_local_stages)
    n, k, B = cfg["n"], cfg["k"], cfg["b"]
    full = bench.make_catalog_shard(cfg, 0, n, cuda_device)
    qs = [bench.make_queries(cfg, cuda_device), _queries(cfg, 12345, cuda_device)]
    excl = None
    if excl_per_query:
        rng = np.random.default_rng(3)
        excl = [np.sort(rng.choice(n, excl_per_query, replace=False)) for _ in range(B)]
    torch.cuda.synchronize(cuda_device)
    if check_plan is not None:
        check_plan(n, B)

    def body(rank, cat, coll):
        outs = []
        for m in (1, 2):   # batch 0 alone; then batches 0 and 1 in flight (returns batch 1)
            it = iter(qs[:m])
            outs.append(run_sharded_steps(
                lambda: score_topk_sharded_local_stages(cat, k, queries=next(it),
                                                        exclude=excl, collectives=coll), m))
        torch.cuda.synchronize(cuda_device)
        return outs

    def body_c(rank, cat, coll):
        # the C ABI's step (ebt_cosine_topk_sharded_submit / _finish / _wait) over the same
        # thread exchange: batch 0 alone, then batches 0 and 1 in flight (returns batch 1)
        def gather(recv, send):
            recv.copy_(coll.all_gather(send).reshape(-1))
        eng = ShardedTopk(cat, k, B, TorchGatherComm(rank, WORLD, gather=gather), slots=slots)
        outs = [tuple(t.clone() for t in eng(queries=qs[0], exclude=excl))]
        if slots >= 2:
            eng.submit(0, queries=qs[0], exclude=excl)
            eng.submit(1, queries=qs[1], exclude=excl)
            eng.finish(0)
            eng.finish(1)
            eng.wait(0)
            outs.append(tuple(t.clone() for t in eng.wait(1)))
        torch.cuda.synchronize(cuda_device)
        return outs
    _log(f"{n} x {cfg['d']} {cfg['dtype']}, B={B}, k={k}: {WORLD} thread ranks, {path} path")
    res = _run_sharded(full, WORLD, body if path == "python" else body_c)
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    _log("sharded batches done; single-GPU reference")
    whole = ebt.Catalog(full)
    for i, q in enumerate(qs[:len(res[0])]):
        s_ref, r_ref = ebt.score_topk(whole, k, queries=q, exclude=excl)
        for rank in range(WORLD):
            s, r = res[rank][i]
            assert torch.equal(r, r_ref), f"batch {i}: rank {rank}'s merged rows differ"
            assert torch.equal(s, s_ref), f"batch {i}: rank {rank}'s merged scores differ"
        _check_properties(s_ref, r_ref, n, excl)
    del whole
    # sampled queries of the first batch vs the host float64 oracle over the whole catalog
    s, r = res[0][0]
    idx = np.unique(np.linspace(0, B - 1, n_sample).round().astype(np.int64))
    qh = qs[0][torch.from_numpy(idx).to(cuda_device)].float().cpu().numpy()
    ex = None if excl is None else [excl[i] for i in idx]
    _log(f"host float64 oracle on {len(idx)} queries")
    s_o, r_o = R.cosine_topk_stream(qh, device_blocks(full), k, ex, workers=8)
    _log("oracle done")
    np.testing.assert_array_equal(r.cpu().numpy()[idx], r_o)
    np.testing.assert_allclose(s.cpu().numpy()[idx], s_o, rtol=0, atol=SCORE_ATOL)


@pytest.mark.parametrize("path", ["python", "capi"])
def test_c3_eight_ranks_shared_threshold(cuda_device, path):
    """C3 on 8 ranks: 125K-row shards, the shared screening threshold, exclusions; the Python
    pipeline and the C ABI's step."""
    import bench
    from robot_ebert_amd.distributed import shard_range, shared_sample_tiles
    from robot_ebert_amd.search import pad_batch

    def plan(n, B):
        assert shared_sample_tiles(n, WORLD, pad_batch(B)) > 0
        assert shard_range(n, WORLD - 1, WORLD)[1] == n
    _sharded_at_scale(cuda_device, dict(bench.CONFIGS["C3"]), 32, excl_per_query=128,
                      check_plan=plan, path=path)


@pytest.mark.parametrize("path", ["python", "capi"])
def test_c4_whole_catalog_eight_ranks(cuda_device, path):
    """C4: the whole 10M x 768 bf16 catalog as 8 shards of 1.25M rows, 8192 queries, top-100."""
    import bench
    from robot_ebert_amd.distributed import shared_sample_tiles
    from robot_ebert_amd.search import pad_batch

    def plan(n, B):
        assert shared_sample_tiles(n, WORLD, pad_batch(B)) == 0   # per-shard screens
    _sharded_at_scale(cuda_device, dict(bench.CONFIGS["C4"]), 32, check_plan=plan, path=path)


@pytest.mark.parametrize("path", ["python", "capi"])
def test_c5_batch_and_k_eight_ranks(cuda_device, path):
    """C5's batch and k (16384 queries, top-1000: k' = 1256, the floor-only branch with the
    block merge) on 8 shards of 1M x 1536 f16."""
    import bench
    import robot_ebert_amd as ebt
    from robot_ebert_amd.search import MERGE_WAVE_KMAX, default_kprime
    cfg = dict(bench.CONFIGS["C5"], n=8 * 1_000_000)

    def plan(n, B):
        shard = ebt.Catalog(torch.zeros((256, cfg["d"]), dtype=torch.float16,
                                        device=cuda_device))
        assert default_kprime(shard, cfg["k"]) > MERGE_WAVE_KMAX
    # the C path with one batch (8 ranks x a 16384-query workspace of ~8 GB each)
    _sharded_at_scale(cuda_device, cfg, 32, check_plan=plan, path=path, slots=1)


def test_c5_batch_and_k_eight_ranks_capi_two_slots(cuda_device):
    """The C ABI's batches-in-flight mode at C5's batch and k: two slots
    (batch 0 alone, then batches 0 and 1 submitted before either finishes) on 8 thread ranks of
    250K x 1536 f16 each -- the 1M-row shards of the test above need ~23 GiB of workspace per
    slot and rank, more than one GPU holds for 8 ranks x 2 slots."""
    import bench
    import robot_ebert_amd as ebt
    from robot_ebert_amd.search import MERGE_WAVE_KMAX, default_kprime
    cfg = dict(bench.CONFIGS["C5"], n=8 * 250_000)

    def plan(n, B):
        shard = ebt.Catalog(torch.zeros((256, cfg["d"]), dtype=torch.float16,
                                        device=cuda_device))
        assert default_kprime(shard, cfg["k"]) > MERGE_WAVE_KMAX   # k' = 1256: block merges
    _sharded_at_scale(cuda_device, cfg, 16, check_plan=plan, path="capi", slots=2)
