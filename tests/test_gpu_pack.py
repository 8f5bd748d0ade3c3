"""GPU: the compact exchange of the row-sharded step (include/ebert.h ebt_shard_pack,
ebt_merge_packed, ebt_floor_pack) against numpy and ebt_merge_topk over the full lists.

The packed merge must give the same global top-k as the full merge whenever every global top-k
entry is at or above the floor (what the catalog-wide floor guarantees), flag a batch whose
packed entries did not fit, and the floor pack must send each shard's w largest approx values
(its list may be partitioned, not sorted). Reference: /root/reference/src/backend/app/lib.py:55
(sort + [:k]) restated across shards.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from robot_ebert_amd import _lib as L
    return L


def sorted_lists(rng, R, B, k, n_real, ties=False):
    """[R, B, k] per-shard lists sorted (score desc, row asc), the first n_real[r, b] real,
    the rest padding (row -1, score NaN); rows disjoint across shards."""
    s = np.full((R, B, k), np.nan)
    r = np.full((R, B, k), -1, dtype=np.int64)
    for a in range(R):
        for b in range(B):
            m = int(n_real[a, b])
            v = rng.standard_normal(m)
            if ties:
                v = np.round(v * 4) / 4
            rows = rng.choice(1_000_000, m, replace=False) * R + a
            o = np.lexsort((rows, -v))
            s[a, b, :m], r[a, b, :m] = v[o], rows[o]
    return s, r


@pytest.mark.parametrize("R,B,k,ties", [(8, 300, 100, False), (8, 64, 100, True),
                                        (3, 100, 1000, False), (2, 17, 7, True)])
def test_pack_merge_equals_full_merge(cuda_device, R, B, k, ties):
    L = _lib()
    dev = cuda_device
    rng = np.random.default_rng(R * 1000 + k)
    n_real = rng.integers(0, k + 1, size=(R, B))
    n_real[:, :3] = k
    s, r = sorted_lists(rng, R, B, k, n_real, ties)
    # the floor: the k-th best over all shards minus a margin (some below it are sent too)
    flat = np.where(r >= 0, s, -np.inf).transpose(1, 0, 2).reshape(B, R * k)
    kth = -np.sort(-flat, axis=1)[:, k - 1]
    floor = np.where(np.isfinite(kth), kth - 0.05, -np.inf)
    floor[5] = -np.inf
    st = torch.cuda.current_stream(dev).cuda_stream
    gs, gr = torch.from_numpy(s).to(dev), torch.from_numpy(r).to(dev)
    full_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    full_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    L.call("ebt_merge_topk", L.ptr(gs), L.ptr(gr), R, B, k, L.ptr(full_s), L.ptr(full_r), st)
    cap = L.load().ebt_shard_pack_cap(B, k, R, 1 << 30)
    assert cap == B * min(k, -(-3 * k // (2 * R)) + 8)
    nbytes = L.load().ebt_shard_pack_bytes(B, cap)
    recv = torch.zeros(R * nbytes, dtype=torch.uint8, device=dev)
    tf = torch.from_numpy(floor).to(dev)
    counts, per_query = [], np.zeros(B, dtype=np.int64)
    for a in range(R):
        L.call("ebt_shard_pack", L.ptr(gs[a].contiguous()), L.ptr(gr[a].contiguous()), B, k,
               L.ptr(tf), cap, L.ptr(recv[a * nbytes:]), st)
        # header (0.3.2): u32 start[B], u32 len[B]; ebt_shard_pack's starts are the prefix sum
        hdr = recv[a * nbytes:a * nbytes + 8 * B].view(torch.int32).cpu().numpy()
        start, ln = hdr[:B], hdr[B:]
        want = ((r[a] >= 0) & (s[a] >= floor[:, None])).sum(1)
        np.testing.assert_array_equal(ln, want)
        np.testing.assert_array_equal(start, np.concatenate([[0], np.cumsum(want)[:-1]]))
        counts.append(int(want.sum()))
        per_query += want
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    inc = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("ebt_merge_packed", L.ptr(recv), R, B, k, cap, L.ptr(out_s), L.ptr(out_r), L.ptr(inc),
           st)
    # a rank over its cap, or (0.3.3) a query over the merge's room min(R k, 2 k + 256)
    overflow = max(counts) > cap or int(per_query.max()) > min(R * k, 2 * k + 256)
    assert bool(inc.item()) == overflow
    if not overflow:
        assert torch.equal(out_r, full_r)
        m = full_r >= 0
        assert torch.equal(out_s[m], full_s[m])
        assert torch.isnan(out_s[~m]).all()


def test_pack_overflow_flags(cuda_device):
    """A shard with more entries above the floor than its cap: the batch is flagged."""
    L = _lib()
    dev = cuda_device
    R, B, k = 4, 64, 50
    rng = np.random.default_rng(7)
    s, r = sorted_lists(rng, R, B, k, np.full((R, B), k))
    st = torch.cuda.current_stream(dev).cuda_stream
    cap = L.load().ebt_shard_pack_cap(B, k, R, 1 << 30)
    nbytes = L.load().ebt_shard_pack_bytes(B, cap)
    recv = torch.zeros(R * nbytes, dtype=torch.uint8, device=dev)
    gs, gr = torch.from_numpy(s).to(dev), torch.from_numpy(r).to(dev)
    for a in range(R):   # no floor: all 50 entries per query, 27 fit on average
        L.call("ebt_shard_pack", L.ptr(gs[a].contiguous()), L.ptr(gr[a].contiguous()), B, k,
               None, cap, L.ptr(recv[a * nbytes:]), st)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    inc = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("ebt_merge_packed", L.ptr(recv), R, B, k, cap, L.ptr(out_s), L.ptr(out_r), L.ptr(inc),
           st)
    assert inc.item() == 1


@pytest.mark.parametrize("per_rank,flagged", [(57, False), (58, True), (100, True)])
def test_pack_merge_room(cuda_device, per_rank, flagged):
    """The packed merge holds min(R k, 2 k + 256) entries per query (R 8, k 100: 456): with a
    cap that every rank's entries fit, 8 x 57 = 456 entries per query merge exactly as the full
    merge does, 8 x 58 = 464 flag the batch incomplete (the caller's full exchange)."""
    L = _lib()
    dev = cuda_device
    R, B, k = 8, 16, 100
    rng = np.random.default_rng(per_rank)
    s, r = sorted_lists(rng, R, B, k, np.full((R, B), per_rank))
    st = torch.cuda.current_stream(dev).cuda_stream
    gs, gr = torch.from_numpy(s).to(dev), torch.from_numpy(r).to(dev)
    full_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    full_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    L.call("ebt_merge_topk", L.ptr(gs), L.ptr(gr), R, B, k, L.ptr(full_s), L.ptr(full_r), st)
    cap = B * k                                   # every rank's entries fit: only the room limits
    nbytes = L.load().ebt_shard_pack_bytes(B, cap)
    recv = torch.zeros(R * nbytes, dtype=torch.uint8, device=dev)
    for a in range(R):   # no floor: every real entry is sent
        L.call("ebt_shard_pack", L.ptr(gs[a].contiguous()), L.ptr(gr[a].contiguous()), B, k,
               None, cap, L.ptr(recv[a * nbytes:]), st)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    inc = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("ebt_merge_packed", L.ptr(recv), R, B, k, cap, L.ptr(out_s), L.ptr(out_r), L.ptr(inc),
           st)
    assert bool(inc.item()) == flagged
    if not flagged:
        assert torch.equal(out_r, full_r)
        assert torch.equal(out_s, full_s)


@pytest.mark.parametrize("ld,k_eff,w", [(200, 100, 27), (1256, 1000, 196), (40, 40, 40),
                                        (120, 100, 8), (64, 0, 5), (300, 30, 50)])
def test_floor_pack_selects_w_largest(cuda_device, ld, k_eff, w):
    L = _lib()
    dev = cuda_device
    B = 37
    rng = np.random.default_rng(ld + w)
    v = (np.round(rng.standard_normal((B, ld)) * 8) / 8).astype(np.float32)  # ties
    v[1, :] = -np.inf
    v[2, ::3] = np.nan
    v[3, 5:] = -np.inf                                                        # few valid
    eps = rng.random(B).astype(np.float32)
    out = torch.empty((B, w + 1), dtype=torch.float32, device=dev)
    vd, ed = torch.from_numpy(v).to(dev), torch.from_numpy(eps).to(dev)
    L.call("ebt_floor_pack", L.ptr(vd), ld, B, k_eff, w, L.ptr(ed), L.ptr(out),
           torch.cuda.current_stream(dev).cuda_stream)
    o = out.cpu().numpy()
    np.testing.assert_array_equal(o[:, w], eps)
    n = min(k_eff, ld)
    for b in range(B):
        x = v[b, :n]
        x = x[np.isfinite(x) | (x == np.inf)]
        want = -np.sort(-x)[:w]
        want = np.concatenate([want, np.full(w - len(want), -np.inf, np.float32)])
        np.testing.assert_array_equal(-np.sort(-o[b, :w]), want)
