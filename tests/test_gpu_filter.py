"""The filter epilogue of the screening GEMM (screen_gemm.hip: column test, compacted staging of
the flagged (lane, query column) pairs, rounds of 16 per wave) against the store epilogue of
the same kernel: for every (query, 256-row group) whose hits fit the slots, the hit set is
EXACTLY {(f2key(s) << 32) | ~row : s >= thr} of the stored scores (both epilogues compute
fl(fl(a * qs) * cs)), the group count is exact, and a group with more hits than slots sets the
query's overflow flag. Hit densities from a few per wave to ~40 % of all scores (every lane of
every wave flagged: 16 staging rounds), with and without row scales (the lowered-threshold
column test), a ragged last tile and an odd K-tile count."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _key(v):
    v = np.asarray(v, dtype=np.float32) + np.float32(0.0)
    u = v.view(np.uint32).astype(np.uint64)
    k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    bad = np.isnan(v) | (v == -np.inf)
    return np.where(bad, 0, k).astype(np.uint64)


@pytest.mark.parametrize("density", [0.002, 0.05, 0.4])
@pytest.mark.parametrize("d,scaled", [(128, False), (192, True), (256, True), (192, False)])
def test_filter_matches_store(cuda_device, density, d, scaled):
    from robot_ebert_amd import _lib as L
    dev = cuda_device
    B, N, base = 512, 3 * 1024 + 77, 11
    g = torch.Generator(device=dev).manual_seed(17 + d)
    q = torch.randn((B, d), generator=g, device=dev).half()
    c = torch.randn((N, d), generator=g, device=dev).half()
    qs = (torch.rand(B, generator=g, device=dev) + 0.5).contiguous()
    cs = ((torch.rand(((N + 127) // 128) * 128, generator=g, device=dev) + 0.5).contiguous()
          if scaled else None)
    st = L.stream_of(dev)
    code = L.DTYPE_CODE[torch.float16]
    ld = (N + 3) // 4 * 4
    S = torch.full((B, ld), float("nan"), device=dev)
    L.call("ebt_screen_scores", L.ptr(q), B, L.ptr(c), N, d, d, code, L.ptr(qs),
           L.ptr(cs) if scaled else None, L.ptr(S), ld, st)
    S = S[:, :N]
    thr = torch.quantile(S[:, :2048], 1.0 - density, dim=1).contiguous()
    G = int(L.load().ebt_filter_group_rows(B))
    assert G == 256
    groups = (N + G - 1) // G
    slots = 128
    cand = torch.zeros((B, groups * slots), dtype=torch.int64, device=dev)
    counts = torch.zeros((B, groups), dtype=torch.uint8, device=dev)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    L.call("ebt_screen_filter", L.ptr(q), B, L.ptr(c), N, d, d, code, L.ptr(qs),
           L.ptr(cs) if scaled else None, L.ptr(thr), L.ptr(cand), groups * slots, slots,
           L.ptr(counts), groups, L.ptr(ovf), base, st)
    torch.cuda.synchronize(dev)

    s = S.cpu().numpy()
    t = thr.cpu().numpy()
    hit = s >= t[:, None]
    pad = groups * G - N
    hitp = np.pad(hit, ((0, 0), (0, pad)))
    want_cnt = hitp.reshape(B, groups, G).sum(-1)
    rows = np.arange(N, dtype=np.uint64) + np.uint64(base)
    comp = (_key(s) << np.uint64(32)) | ((~rows) & np.uint64(0xFFFFFFFF))[None, :]
    comp = np.where(hit, comp, np.uint64(0))
    compp = np.pad(comp, ((0, 0), (0, pad))).reshape(B, groups, G)
    want_sorted = np.sort(compp, axis=-1)[:, :, ::-1][:, :, :slots]   # hits first, descending

    got_cnt = counts.cpu().numpy().astype(np.int64)
    got = cand.cpu().numpy().view(np.uint64).reshape(B, groups, slots)
    live = np.arange(slots)[None, None, :] < np.minimum(got_cnt, slots)[:, :, None]
    got_sorted = np.sort(np.where(live, got, np.uint64(0)), axis=-1)[:, :, ::-1]

    fits = want_cnt <= slots
    assert np.array_equal(got_cnt[fits], want_cnt[fits])
    assert np.array_equal(got_cnt[~fits], np.minimum(want_cnt[~fits], 255))
    assert np.array_equal(got_sorted[fits], want_sorted[fits]), "hit sets differ"
    ov = ovf.cpu().numpy() != 0
    assert np.array_equal(ov, (~fits).any(axis=1))
    mean_hits = float(want_cnt.sum()) / B
    print(f"d={d} scaled={scaled} density={density}: {mean_hits:.0f} hits per query, "
          f"{int((~fits).sum())} overflowing groups")


@pytest.mark.parametrize("lists", ["full", "shuffle", "ragged"])
@pytest.mark.parametrize("R,k", [(2, 100), (8, 100), (8, 1000), (16, 1000), (3, 4096), (64, 128),
                                 (2, 1), (5, 3), (100, 20), (1024, 8)])
def test_merge_topk_any_rank_count(cuda_device, R, k, lists):
    """ebt_merge_topk (the post-all-gather merge): sorted lists with R * k <= 8192 by co-ranks,
    above that in bitonic rounds that keep the running top k, unsorted lists (shuffle) by the
    bitonic network; equals a numpy (score desc, row asc) merge, with ties across ranks, empty
    (-1) slots and NaN scores sorting last; ragged: each list padded (-1) after a random number
    of entries, 0 to k, as the per-shard lists are after the floor cut (C3/8: ~18 of 100)."""
    from robot_ebert_amd import _lib as L
    dev = cuda_device
    B = 6
    shuffle = lists == "shuffle"
    rng = np.random.default_rng(R * 7 + k)
    s = np.round(rng.standard_normal((R, B, k)), 2)          # many exact ties across ranks
    rows = rng.permutation(R * B * k * 2)[:R * B * k].reshape(R, B, k).astype(np.int64)
    s[:, :, -3:] = np.nan
    rows[:, :, -1] = -1
    s[:, 0, :] = 0.5                                          # one query all tied
    if lists == "ragged":
        V = rng.integers(0, k + 1, (R, B))
        V[:, 1] = max(1, k // (2 * R))                        # every list short, a few valid
        V[:, 2] = 0                                           # nothing valid at all
        for r in range(R):
            for b in range(B):
                rows[r, b, V[r, b]:] = -1
    # each rank's list sorted (score desc, row asc), NaN / -1 last
    for r in range(R):
        for b in range(B):
            key = np.where(rows[r, b] < 0, -np.inf, np.where(np.isnan(s[r, b]), -np.inf, s[r, b]))
            o = np.lexsort((np.where(rows[r, b] < 0, np.iinfo(np.int64).max, rows[r, b]), -key))
            if shuffle and r == R // 2:
                o = rng.permutation(o)
            s[r, b], rows[r, b] = s[r, b][o], rows[r, b][o]
    ts = torch.tensor(s, device=dev)
    tr = torch.tensor(rows, device=dev)
    os_ = torch.empty((B, k), dtype=torch.float64, device=dev)
    or_ = torch.empty((B, k), dtype=torch.int64, device=dev)
    L.call("ebt_merge_topk", L.ptr(ts), L.ptr(tr), R, B, k, L.ptr(os_), L.ptr(or_),
           L.stream_of(dev))
    torch.cuda.synchronize(dev)
    got_s, got_r = os_.cpu().numpy(), or_.cpu().numpy()
    for b in range(B):
        fs, fr = s[:, b].ravel(), rows[:, b].ravel()
        ok = fr >= 0
        key = np.where(np.isnan(fs[ok]), -np.inf, fs[ok])
        o = np.lexsort((fr[ok], -key))[:k]
        want_r = fr[ok][o]
        want_s = np.where(np.isnan(fs[ok][o]), -np.inf, fs[ok][o])
        m = len(want_r)
        assert np.array_equal(got_r[b, :m], want_r), b
        assert np.array_equal(got_s[b, :m], want_s), b
        assert (got_r[b, m:] == -1).all()
