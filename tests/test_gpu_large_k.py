"""k beyond the screen's k' range (min(k, n) > 4096): the full-sort path (large_k.hip) --
every score in float64, a descending (score, row) merge sort cut at k, the first k -- against the float64
oracle (oracle/restatement.py: lib.py:51-55 restated): rows bit-exact in (score desc, row asc)
order, scores within 1e-12, NaN / -1 past the valid rows (k > n, exclusions), exact duplicate
rows ordered by row, dense / liked queries, f32 / bf16 catalogs. The reference's pandas [:k]
takes any k; so does ebt_cosine_topk."""
import numpy as np
import pytest
import torch

from oracle import restatement as R

pytestmark = pytest.mark.gpu


def _catalog(n, d, seed, dup=()):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((n, d))
    for a, b in dup:          # exact duplicates: tied scores, ordered by row
        c[b] = c[a]
    return c


def _check(s, r, s_ref, r_ref):
    assert np.array_equal(r, r_ref), np.nonzero((r != r_ref).any(axis=1))
    valid = r_ref >= 0
    assert np.all(np.isnan(s[~valid]))
    assert np.max(np.abs(s[valid] - s_ref[valid])) <= 1e-12


@pytest.mark.parametrize("k", [5000, 12000])
def test_large_k_dense_with_exclusions(cuda_device, k):
    import robot_ebert_amd as ebt
    n, d, B = 9000, 48, 5
    c = _catalog(n, d, 7, dup=[(10, 8000), (11, 20), (4000, 4001)])
    rng = np.random.default_rng(8)
    q = rng.standard_normal((B, d))
    q[2] = c[10]                                   # a query equal to a duplicated row
    excl = [sorted(rng.choice(n, 300, replace=False).tolist()) for _ in range(B)]
    excl[1] = []
    cat = ebt.Catalog(torch.tensor(c, dtype=torch.float32, device=cuda_device))
    c32 = c.astype(np.float32).astype(np.float64)   # the catalog the GPU holds
    q32 = q.astype(np.float32).astype(np.float64)
    s, r = ebt.score_topk(cat, k, queries=torch.tensor(q32, dtype=torch.float32,
                                                       device=cuda_device), exclude=excl)
    s_ref, r_ref = R.cosine_topk(q32, c32, k, exclude=excl)
    _check(s.cpu().numpy(), r.cpu().numpy(), s_ref, r_ref)
    assert (r.cpu().numpy()[1] >= 0).sum() == min(k, n)
    assert (r.cpu().numpy()[0] >= 0).sum() == min(k, n - 300)


def test_large_k_liked_bf16(cuda_device):
    import robot_ebert_amd as ebt
    n, d, k = 6000, 64, 5500
    c = _catalog(n, d, 9, dup=[(5, 5999)])
    cb = torch.tensor(c, dtype=torch.float32).to(torch.bfloat16)
    c64 = cb.double().numpy()
    liked = [[5, 77, 300], [1234], [5999, 5]]
    excl = [sorted(set(x) | {100, 200}) for x in liked]
    cat = ebt.Catalog(cb.to(cuda_device))
    s, r = ebt.score_topk(cat, k, liked=liked, exclude=excl)
    s_ref, r_ref = R.liked_topk(c64, liked, k, exclude=excl)
    _check(s.cpu().numpy(), r.cpu().numpy(), s_ref, r_ref)


def test_large_k_many_runs_and_groups(cuda_device):
    """The hand-written sort (round 6) past one LDS run and one query group: n = 70 000 rows are
    35 sorted runs and 6 merge passes, the later ones cut at k; 70 queries are two groups of the
    key budget's at most 64; many exact duplicates (tied scores across runs) ordered by row;
    an all-excluded-but-few query leaves NaN / -1 slots."""
    import robot_ebert_amd as ebt
    n, d, B, k = 70_000, 16, 70, 4500
    rng = np.random.default_rng(11)
    c = rng.standard_normal((n, d))
    src = rng.integers(0, n, size=3000)
    dst = rng.integers(0, n, size=3000)
    c[dst] = c[src]                                   # ties spread over every run
    q = rng.standard_normal((B, d))
    q[3] = c[src[0]]
    excl = [sorted(rng.choice(n, 50, replace=False).tolist()) for _ in range(B)]
    excl[7] = list(range(0, n - 1000))                # only 1000 candidates left
    cat = ebt.Catalog(torch.tensor(c, dtype=torch.float32, device=cuda_device))
    c32 = c.astype(np.float32).astype(np.float64)
    q32 = q.astype(np.float32).astype(np.float64)
    s, r = ebt.score_topk(cat, k, queries=torch.tensor(q32, dtype=torch.float32,
                                                       device=cuda_device), exclude=excl)
    s_ref, r_ref = R.cosine_topk(q32, c32, k, exclude=excl)
    _check(s.cpu().numpy(), r.cpu().numpy(), s_ref, r_ref)
    assert (r.cpu().numpy()[7] >= 0).sum() == 1000
