"""GPU parity at the BASELINE GPU workloads (BASELINE.json configs C2-C5), against the oracle.

Each test builds the bench's own seeded catalog (bench.make_catalog_shard: the same rows bench.py
times) and query batch on the device, runs the product path (robot_ebert_amd.score_topk over the
C ABI) on the FULL batch, and checks
  * sampled queries against the host float64 oracle (oracle.restatement.cosine_topk_stream: the
    catalog streamed to the host in row blocks, upcast to float64 there) -- rows bit-exact,
    scores within 1e-12 (north_star: 1e-5);
  * every query of the batch against torch float64 on the device (a cross-check of the same
    arithmetic, not the oracle) -- rows bit-exact, scores within 1e-12;
  * properties of every query: scores non-increasing, rows unique and inside the shard, no
    excluded row, |score| <= 1.
Reference: /root/reference/src/backend/app/lib.py:51-55 (cosine_similarity + mean + exclusion
+ sort + [:k]).

C2 and C3 run at their full size; C4 and C5 are 8-GPU configurations, so they run at the
per-rank work of an 8-way row shard (rank 3's rows, global row ids through row_offset). The
single-GPU full-size C4 / C5 runs are bench lines (bench.py --config C4 / C5).
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import restatement as R

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SCORE_ATOL = 1e-12


def _bench():
    import bench
    return bench


def device_blocks(emb: torch.Tensor, block: int = 1 << 17):
    """Row blocks of a device matrix as host float32 arrays (f16 / bf16 -> f32 is exact; the
    float64 arithmetic is the oracle's, on the host)."""
    for r0 in range(0, emb.shape[0], block):
        yield r0, emb[r0:r0 + block].float().cpu().numpy()


def device_f64_topk(emb: torch.Tensor, q: torch.Tensor, k: int, excl=None, qblock: int = 2048,
                    block: int = 1 << 17):
    """Every query's exact top-k in float64 on the device: sklearn's normalise (norm < 10 eps
    -> 1), scores q_hat . c / |c|, (score desc, row asc). Keeps k + 16 per query between blocks."""
    dev = q.device
    B = q.shape[0]
    eps = torch.finfo(torch.float64).eps
    q64 = q.double()
    qn = q64.norm(dim=1, keepdim=True)
    q64 = q64 / torch.where(qn < 10 * eps, torch.ones_like(qn), qn)
    keep = k + 16
    best_s = torch.full((B, 0), float("-inf"), dtype=torch.float64, device=dev)
    best_r = torch.empty((B, 0), dtype=torch.int64, device=dev)
    for c0 in range(0, emb.shape[0], block):
        c = emb[c0:c0 + block].double()
        g = c.norm(dim=1)
        g = torch.where(g < 10 * eps, torch.ones_like(g), g)
        ns, nr = [], []
        for b0 in range(0, B, qblock):
            sc = (q64[b0:b0 + qblock] @ c.T) / g
            if excl is not None:
                eq, er = excl
                m = (eq >= b0) & (eq < b0 + qblock) & (er >= c0) & (er < c0 + c.shape[0])
                sc[eq[m] - b0, er[m] - c0] = float("-inf")
            s2 = torch.cat([best_s[b0:b0 + qblock], sc], 1)
            rows = torch.arange(c0, c0 + c.shape[0], device=dev).expand(s2.shape[0], -1)
            r2 = torch.cat([best_r[b0:b0 + qblock], rows], 1)
            ts, ti = torch.topk(s2, min(keep, s2.shape[1]), dim=1)
            ns.append(ts)
            nr.append(torch.gather(r2, 1, ti))
            del sc, s2, r2
        best_s, best_r = torch.cat(ns), torch.cat(nr)
        del c
    o = torch.argsort(best_r, dim=1)
    best_s, best_r = torch.gather(best_s, 1, o), torch.gather(best_r, 1, o)
    o = torch.argsort(-best_s, dim=1, stable=True)
    return torch.gather(best_s, 1, o)[:, :k], torch.gather(best_r, 1, o)[:, :k]


def run_workload(cuda_device, config: str, rank: int = 0, world: int = 1, n_sample: int = 64,
                 excl_per_query: int = 0, full_device_check: bool = True, **override):
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import shard_range
    bench = _bench()
    cfg = dict(bench.CONFIGS[config], **override)
    begin, end = shard_range(cfg["n"], rank, world)
    emb = bench.make_catalog_shard(cfg, begin, end, cuda_device)
    q = bench.make_queries(cfg, cuda_device)
    B, k = cfg["b"], cfg["k"]
    excl_lists, excl_dev = None, None
    if excl_per_query:
        rng = np.random.default_rng(3)
        excl_lists = [np.sort(rng.choice(end - begin, excl_per_query, replace=False)) + begin
                      for _ in range(B)]
        eq = torch.from_numpy(np.repeat(np.arange(B), excl_per_query)).to(cuda_device)
        er = torch.from_numpy(np.concatenate(excl_lists) - begin).to(cuda_device)
        excl_dev = (eq, er)
    cat = ebt.Catalog(emb, row_offset=begin, n_global=cfg["n"])
    s, r = ebt.score_topk(cat, k, queries=q, exclude=excl_lists)
    torch.cuda.synchronize(cuda_device)
    assert s.shape == (B, k) and r.shape == (B, k)

    # properties of every query
    sn, rn = s.cpu().numpy(), r.cpu().numpy()
    assert np.all(np.isfinite(sn)) and np.all(rn >= begin) and np.all(rn < end)
    assert np.all(np.diff(sn, axis=1) <= 0)
    assert np.all(np.abs(sn) <= 1 + 1e-12)
    rs = np.sort(rn, axis=1)
    assert np.all(np.diff(rs, axis=1) > 0), "duplicate rows in a query's top-k"
    if excl_lists is not None:
        for b in range(0, B, 7):
            assert not np.isin(rn[b], excl_lists[b]).any()

    # sampled queries vs the host float64 oracle (catalog streamed in row blocks)
    idx = np.unique(np.linspace(0, B - 1, n_sample).round().astype(np.int64))
    qh = q[torch.from_numpy(idx).to(cuda_device)].float().cpu().numpy()
    ex = None if excl_lists is None else [excl_lists[i] - begin for i in idx]
    s_ref, r_ref = R.cosine_topk_stream(qh, device_blocks(emb), k, ex, workers=8)
    np.testing.assert_array_equal(rn[idx], r_ref + begin)
    np.testing.assert_allclose(sn[idx], s_ref, rtol=0, atol=SCORE_ATOL)

    # every query vs torch float64 on the device
    if full_device_check:
        ds, dr = device_f64_topk(emb, q, k, excl_dev)
        assert torch.equal(dr + begin, r), "device float64 top-k rows differ"
        assert (ds - s).abs().max().item() <= SCORE_ATOL
    return len(idx)


def test_c2_full_with_exclusions(cuda_device):
    """C2: 100K x 768 bf16, 1024 queries, top-100, 128 excluded rows per query."""
    run_workload(cuda_device, "C2", n_sample=256, excl_per_query=128)


def test_c3_full(cuda_device):
    """C3 (headline): 1M x 1536 f32, 4096 queries, top-100."""
    run_workload(cuda_device, "C3", n_sample=64)


def test_c4_per_rank_shard(cuda_device):
    """C4 per-rank work: rank 3 of 8 of the 10M x 768 bf16 catalog (1.25M rows), 8192 queries."""
    run_workload(cuda_device, "C4", rank=3, world=8, n_sample=32)


def test_c5_per_rank_shard(cuda_device):
    """C5 per-rank work: rank 5 of 8 of the 50M x 1536 f16 catalog (6.25M rows), 16384 queries,
    top-1000."""
    run_workload(cuda_device, "C5", rank=5, world=8, n_sample=32)


def test_c5_small_batch_many_groups(cuda_device):
    """C5's k (top-1000, k' = 1256) with a small batch (1024 queries) over 4.5M rows: the
    speculative screen's segment then spans more 256-row groups than one block merge's LDS
    indexes (16383 at k' = 1256, select_topk.hip merge_block_max_groups); the segment is
    clamped / merged in parts instead of failing."""
    run_workload(cuda_device, "C5", n_sample=16, n=4_500_000, b=1024, full_device_check=False)


@pytest.mark.parametrize("spread", [0.02, 0.2])
def test_clustered_catalog_reruns_stay_exact(cuda_device, spread):
    """the speculative screen's later segments are sized for (k + k') / 2 kept rows
    per r0 rows (api.hip run_screen_spec); on a clustered, near-duplicate-heavy catalog a
    segment's hits may overflow the merge, and each overflowed query is rerun unfused. Here:
    64 tight clusters of ~3100 rows each (row = center + spread x noise), queries drawn at the
    centers, so every query has thousands of rows in its k-th score's neighbourhood. The
    answers stay bit-exact against the float64 oracle whatever the rerun rate, which is
    reported (the first pass's certificates: 1 exact, 0 widened, -1 rerun unfused)."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd.search import score_topk_finish, score_topk_submit
    n, d, B, k, C = 200_000, 128, 512, 100, 64
    rng = np.random.default_rng(17)
    centers = rng.standard_normal((C, d))
    x = centers[rng.integers(0, C, n)] + spread * rng.standard_normal((n, d))
    q = centers[rng.integers(0, C, B)] + spread * 0.5 * rng.standard_normal((B, d))
    x32 = x.astype(np.float32)
    q32 = q.astype(np.float32)
    cat = ebt.Catalog(torch.from_numpy(x32).to(cuda_device))
    p = score_topk_submit(cat, k, queries=torch.from_numpy(q32).to(cuda_device))
    s, r = score_topk_finish(p)
    first = p.cert_host[:B].clone()   # the first pass's (the finish waited for them)
    s_ref, r_ref = R.cosine_topk(q32.astype(np.float64), x32.astype(np.float64), k)
    np.testing.assert_array_equal(r.cpu().numpy(), r_ref)
    np.testing.assert_allclose(s.cpu().numpy(), s_ref, rtol=0, atol=1e-12)
    rates = {c: int((first == c).sum()) for c in (1, 0, -1)}
    print(f"\nclustered spread={spread}: first-pass certificates {rates} of {B}")
    assert sum(rates.values()) == B
