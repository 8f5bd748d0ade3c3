"""GPU parity: every kernel and the whole path vs the float64 oracle / golden vectors.

Bar (north_star): top-k index sets bit-exact, scores within 1e-5 (we test 1e-12 against the
float64 oracle, since the exact rescore is float64). All calls go through the C ABI of
include/ebert.h (libebert.so).
"""
import json
import os

import numpy as np
import pytest
import torch

from inputs import COS_CASES, c1_catalog, cos_case_inputs, gaussian
from oracle import restatement as R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TORCH_DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
SCORE_ATOL = 1e-12  # float64 rescore vs float64 oracle (north_star asks 1e-5)


def _ebt():
    import robot_ebert_amd as ebt
    from robot_ebert_amd import _lib
    return ebt, _lib


def _t(x, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev).to(TORCH_DT[dt])


def assert_topk_equal(s, r, s_ref, r_ref, atol=SCORE_ATOL):
    s = s.cpu().numpy() if torch.is_tensor(s) else s
    r = r.cpu().numpy() if torch.is_tensor(r) else r
    np.testing.assert_array_equal(r, r_ref)
    m = r_ref >= 0
    np.testing.assert_allclose(s[m], s_ref[m], rtol=0, atol=atol)
    assert np.all(np.isnan(s[~m]))


# ------------------------------------------------------------------------------ kernels ----
@pytest.mark.parametrize("dt", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("d", [32, 77, 768])
def test_row_norms(cuda_device, dt, d):
    ebt, L = _ebt()
    x = gaussian(11, 1000, d, dt)
    x[3] = 0.0
    xt = _t(x, dt, cuda_device)
    g = torch.empty(1000, dtype=torch.float64, device=cuda_device)
    inv = torch.empty(1000, dtype=torch.float32, device=cuda_device)
    L.call("ebt_row_norms", L.ptr(xt), L.DTYPE_CODE[xt.dtype], 1000, d, d, L.ptr(g), L.ptr(inv),
           L.stream_of(cuda_device))
    ref = R.zero_guard_norms(R.row_norms(x))
    np.testing.assert_allclose(g.cpu().numpy(), ref, rtol=1e-13)
    np.testing.assert_allclose(inv.cpu().numpy(), 1 / ref, rtol=1e-6)
    assert g[3].item() == 1.0


@pytest.mark.parametrize("img", ["f16", "bf16"])
@pytest.mark.parametrize("shape", [(128, 128, 64), (256, 1000, 768), (128, 4133, 192)])
def test_screen_gemm_vs_torch_fp32(cuda_device, img, shape):
    """MFMA screening GEMM vs a plain PyTorch fp32 reference of the same op."""
    ebt, L = _ebt()
    B, N, d = shape
    tdt = TORCH_DT[img]
    g = torch.Generator(device=cuda_device).manual_seed(5)
    q = torch.randn((B, d), generator=g, device=cuda_device).to(tdt)
    c = torch.randn((N, d), generator=g, device=cuda_device).to(tdt)
    qs = torch.rand(B, generator=g, device=cuda_device) + 0.5
    cs = torch.rand(((N + 127) // 128) * 128, generator=g, device=cuda_device) + 0.5
    ld_s = (N + 3) // 4 * 4
    S = torch.full((B, ld_s), float("nan"), device=cuda_device)
    L.call("ebt_screen_scores", L.ptr(q), B, L.ptr(c), N, d, d, L.DTYPE_CODE[tdt], L.ptr(qs),
           L.ptr(cs), L.ptr(S), ld_s, L.stream_of(cuda_device))
    ref = (q.float() @ c.float().T) * qs[:, None] * cs[None, :N]
    got = S[:, :N]
    err = (got - ref).abs().max().item()
    bound = 1e-5 * (q.float().abs() @ c.float().abs().T).max().item() * 4
    assert err <= bound + 1e-4, (err, bound)
    # A = I style check with an asymmetric operand: row/col mapping
    eye = torch.zeros((128, d), dtype=tdt, device=cuda_device)
    for i in range(min(128, d)):
        eye[i, i] = 1
    one = torch.ones(128, device=cuda_device)
    c2 = torch.arange(N * d, device=cuda_device, dtype=torch.float32).reshape(N, d) % 7
    c2 = c2.to(tdt)
    S2 = torch.zeros((128, ld_s), device=cuda_device)
    L.call("ebt_screen_scores", L.ptr(eye), 128, L.ptr(c2), N, d, d, L.DTYPE_CODE[tdt], L.ptr(one),
           None, L.ptr(S2), ld_s, L.stream_of(cuda_device))
    m = min(128, d)
    torch.testing.assert_close(S2[:m, :N], c2.float().T[:m], rtol=0, atol=0)


@pytest.mark.parametrize("dt", ["f32", "f64", "bf16"])
def test_screen_exact_vs_oracle(cuda_device, dt):
    """ebt_screen_exact: float64 cosine rounded once to f32, against the oracle's float64 cosine
    (f32 rounding of |s| <= 1 is <= 2^-25; ragged B/N/d exercise the tile edges)."""
    ebt, L = _ebt()
    B, N, d = 70, 1333, 77
    c = gaussian(21, N, d, dt)
    c[5] = 0.0
    qv = gaussian(22, B, d, "f64")
    ct = _t(c, dt, cuda_device)
    g = torch.empty(N, dtype=torch.float64, device=cuda_device)
    L.call("ebt_row_norms", L.ptr(ct), L.DTYPE_CODE[ct.dtype], N, d, d, L.ptr(g), None,
           L.stream_of(cuda_device))
    q64 = torch.from_numpy(R.normalize_rows(qv)).to(cuda_device)
    ld_s = N + 3
    S = torch.full((B, ld_s), float("nan"), device=cuda_device)
    L.call("ebt_screen_exact", L.ptr(q64), B, d, L.ptr(ct), L.DTYPE_CODE[ct.dtype], d, L.ptr(g), N,
           L.ptr(S), ld_s, L.stream_of(cuda_device))
    ref = R.cosine_similarity(qv, c.astype(np.float64))
    got = S[:, :N].double().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=0, atol=2.0 ** -24)
    assert torch.isnan(S[:, N:]).all()


def test_exact_screen_fallback_near_ties(cuda_device):
    """A cluster of 10000 rows within ~1e-4 of the top score: the f16 screen cannot certify it
    even at k' = 4096, so the query is screened again in float64 -- and must match the oracle."""
    ebt, L = _ebt()
    n, d, k = 60_000, 64, 50
    rng = np.random.default_rng(4)
    q = rng.standard_normal((1, d))
    c = rng.standard_normal((n, d))
    idx = rng.choice(n, 10_000, replace=False)
    c[idx] = q[0] + rng.standard_normal((idx.size, d)) * 1e-2
    cat = ebt.Catalog(_t(c, "f64", cuda_device))
    s, r = ebt.score_topk(cat, k, queries=_t(q, "f64", cuda_device))
    s_ref, r_ref = R.cosine_topk(q, c, k)
    assert_topk_equal(s, r, s_ref, r_ref)


def _key_of(v):
    """The order-preserving u32 key of float32 values (common.h f2key)."""
    v = np.asarray(v, dtype=np.float32) + np.float32(0.0)  # -0 -> +0, as f2key does
    u = v.view(np.uint32).astype(np.uint64)
    k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    bad = np.isnan(v) | (np.asarray(v) == -np.inf)
    return np.where(bad, 0, k).astype(np.uint64)


def _composite(v, rows):
    return ((_key_of(v) << np.uint64(32)) | ((~np.asarray(rows, dtype=np.uint64)) & np.uint64(0xFFFFFFFF)))


@pytest.mark.parametrize("B", [128, 256])
def test_screen_filter_slots(cuda_device, B):
    """ebt_screen_filter: the hits are exactly the scores >= thr (vs a torch fp32 reference of
    the same product; values within 1e-4 of thr are not judged), each in its group's slots,
    with the right group counts; a starved slot count sets ovf."""
    ebt, L = _ebt()
    N, d = 5000, 128
    g = torch.Generator(device=cuda_device).manual_seed(3)
    q = torch.randn((B, d), generator=g, device=cuda_device).half()
    c = torch.randn((N, d), generator=g, device=cuda_device).half()
    qs = torch.ones(B, device=cuda_device)
    ref = (q.float() @ c.float().T)
    thr = torch.quantile(ref[:, :2048], 0.995, dim=1).contiguous()
    G = L.load().ebt_filter_group_rows(B)
    groups = (N + G - 1) // G
    for slots, expect_ovf in [(64, False), (1, True)]:
        cand = torch.zeros((B, groups * slots), dtype=torch.int64, device=cuda_device)
        counts = torch.zeros((B, groups), dtype=torch.uint8, device=cuda_device)
        ovf = torch.zeros(B, dtype=torch.int32, device=cuda_device)
        L.call("ebt_screen_filter", L.ptr(q), B, L.ptr(c), N, d, d, L.DTYPE_CODE[q.dtype],
               L.ptr(qs), None, L.ptr(thr), L.ptr(cand), groups * slots, slots, L.ptr(counts),
               groups, L.ptr(ovf), 7, L.stream_of(cuda_device))
        refn, thrn = ref.cpu().numpy(), thr.cpu().numpy()
        cn, cc = cand.cpu().numpy().view(np.uint64), counts.cpu().numpy()
        if expect_ovf:
            assert (ovf.cpu().numpy() == 1).any()
            continue
        assert not ovf.cpu().numpy().any()
        for b in range(B):
            want = set(np.nonzero(refn[b] >= thrn[b] + 1e-4)[0].tolist())
            maybe = set(np.nonzero(np.abs(refn[b] - thrn[b]) <= 1e-4)[0].tolist())
            got = {}
            for gi in range(groups):
                assert int(cc[b, gi]) <= slots
                for p in range(cc[b, gi]):
                    comp = cn[b, gi * slots + p]
                    row = int((~comp) & np.uint64(0xFFFFFFFF)) - 7
                    assert gi * G <= row < min((gi + 1) * G, N)
                    got[row] = comp
            assert want <= set(got) <= want | maybe
            rows = np.array(sorted(got))
            if rows.size:
                vals = np.array([got[r] >> np.uint64(32) for r in rows], dtype=np.uint64)
                np.testing.assert_allclose(np.array([_key_val(k) for k in vals]), refn[b, rows],
                                           atol=2e-4)


def _key_val(k):
    k = int(k)
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([u], dtype=np.uint32).view(np.float32)[0])


def check_partitioned(gv, gi, ref_v, ref_r, k, kp):
    """A list partitioned at k (include/ebert.h, ebt_merge_hits) against the sorted reference
    (ref_v, ref_r) = the n <= kp best in (value desc, row asc) order."""
    n = len(ref_r)
    assert np.all(gi[n:] == -1) and np.all(np.isneginf(gv[n:]))
    assert sorted(gi[:n].tolist()) == sorted(ref_r.tolist())
    val_of = dict(zip(ref_r.tolist(), ref_v.tolist()))
    np.testing.assert_array_equal(gv[:n], np.array([val_of[r] for r in gi[:n].tolist()],
                                                   np.float32))
    if n == 0:
        return
    kk = min(k, n)
    assert sorted(gi[:kk].tolist()) == sorted(ref_r[:kk].tolist())
    assert gi[kk - 1] == ref_r[kk - 1]
    assert gi[n - 1] == ref_r[n - 1]


@pytest.mark.parametrize("kp,k,hits,groups,shuffle", [
    (40, 20, 30, 7, False), (200, 100, 500, 300, True), (200, 1, 0, 10, False),
    (200, 200, 500, 300, False), (600, 100, 300, 50, True), (40, 40, 30, 7, True),
    # C5's k' with more groups than one block merge's LDS indexes (16383 at k' = 1256): merged
    # in parts (select_topk.hip merge_segment)
    (1256, 1000, 3000, 20000, False), (1256, 1000, 3000, 40000, True),
    # exactly one block merge's group limit at C5's k', and one group more (the first group of
    # a second part): the boundary of the round-4 r4c fault (block merge)
    (1256, 1000, 3000, "max", False), (1256, 1000, 3000, "max+1", True)])
def test_merge_hits_vs_numpy(cuda_device, kp, k, hits, groups, shuffle):
    """ebt_merge_hits: the k' best of (partitioned list + slot hits), exclusions dropped,
    partitioned at k -- ties included -- against numpy on the same composites."""
    ebt, L = _ebt()
    if isinstance(groups, str):
        gmax = int(L.load().ebt_merge_block_max_groups(kp))
        assert gmax > 1000
        groups = gmax + (1 if groups == "max+1" else 0)
    rng = np.random.default_rng(kp + hits + k)
    B, slots = 9, 16
    vals = np.round(rng.standard_normal((B, kp)) * 8) / 8          # ties
    lv = -np.sort(-vals, axis=1).astype(np.float32)
    lr = rng.permutation(100000)[:B * kp].reshape(B, kp) + 200000
    lv[1, kp // 2:] = -np.inf                                        # short list
    lr[1, kp // 2:] = -1
    for b in range(B):                                               # (value desc, row asc)
        o = np.lexsort((np.where(lr[b] < 0, 1 << 40, lr[b]), -lv[b]))
        lv[b], lr[b] = lv[b][o], lr[b][o]
        if shuffle:  # a partitioned input: only the last entry (the k'-th) stays in place
            nv = int((lr[b] >= 0).sum())
            p = np.concatenate([rng.permutation(nv - 1), np.arange(nv - 1, kp)])
            lv[b], lr[b] = lv[b][p], lr[b][p]
    counts = np.zeros((B, (groups + 15) // 16 * 16), np.uint8)
    cand = np.zeros((B, groups * slots), np.uint64)
    hit_v, hit_r = [[] for _ in range(B)], [[] for _ in range(B)]
    for b in range(B):
        gsel = rng.integers(0, groups, hits)
        for gi in gsel:
            if counts[b, gi] >= slots:
                continue
            v = np.float32(np.round(rng.standard_normal() * 8) / 8)
            r = 1_000_000 + gi * 1000 + counts[b, gi]   # disjoint from the list's rows
            cand[b, gi * slots + counts[b, gi]] = _composite(np.array([v]), np.array([r]))[0]
            counts[b, gi] += 1
            hit_v[b].append(v)
            hit_r[b].append(r)
    excl = [sorted(hit_r[b][::3] + [int(lr[b, 0]) + 5]) for b in range(B)]  # some hits excluded
    eo = np.concatenate([[0], np.cumsum([len(e) for e in excl])]).astype(np.int64)
    er = np.concatenate([np.array(e, np.int64) for e in excl]) if eo[-1] else np.zeros(1, np.int64)
    dev = cuda_device
    fv = torch.from_numpy(lv).to(dev)
    fi = torch.from_numpy(lr.astype(np.int64)).to(dev)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    ct = torch.from_numpy(counts).to(dev)
    cd = torch.from_numpy(cand.view(np.int64)).to(dev)
    eot, ert = torch.from_numpy(eo).to(dev), torch.from_numpy(er).to(dev)
    L.call("ebt_merge_hits", L.ptr(fv), L.ptr(fi), B, kp, k, L.ptr(cd), groups * slots, slots,
           L.ptr(ct), counts.shape[1], groups, 0, L.ptr(eot), L.ptr(ert), L.ptr(ovf),
           L.stream_of(dev))
    gv, gi_ = fv.cpu().numpy(), fi.cpu().numpy()
    assert not ovf.cpu().numpy().any()
    for b in range(B):
        ex = set(excl[b])
        hv = [v for v, r in zip(hit_v[b], hit_r[b]) if r not in ex]
        hr = [r for r in hit_r[b] if r not in ex]
        keep = lr[b] >= 0
        allv = np.concatenate([lv[b][keep], np.array(hv, np.float32)])
        allr = np.concatenate([lr[b][keep], np.array(hr, np.int64)])
        o = np.lexsort((allr, -allv))[:kp]
        if kp > 512:  # the block merge: fully sorted
            m = len(o)
            np.testing.assert_array_equal(gi_[b, :m], allr[o])
            np.testing.assert_array_equal(gv[b, :m], allv[o])
            assert np.all(gi_[b, m:] == -1)
        else:
            check_partitioned(gv[b], gi_[b], allv[o], allr[o], k, kp)


def _select_ref(v, k):
    n = v.shape[0]
    keys = np.where(np.isnan(v) | (v == -np.inf), -np.inf, v)
    valid = np.nonzero(keys > -np.inf)[0]
    order = valid[np.lexsort((valid, -keys[valid]))][:k]
    return order


@pytest.mark.parametrize("n,k,segs,odd_ld", [
    (1, 4, 1, False), (3, 8, 1, False), (4097, 100, 1, False), (100000, 256, 1, False),
    (100000, 256, 7, False), (30000, 1000, 2, False), (9000, 4096, 1, False),
    (50001, 200, 1, True), (20000, 300, 3, True)])
def test_select_topk_exact(cuda_device, n, k, segs, odd_ld):
    """Streaming select (select_topk.hip) vs a numpy lexsort: exact rows and values, ties by row,
    -inf / NaN never selected; odd_ld: a row pitch that is not a multiple of 4 (scalar loads)."""
    ebt, L = _ebt()
    rng = np.random.default_rng(n + k)
    B = 6
    v = rng.standard_normal((B, n)).astype(np.float32)
    v[1] = np.round(v[1] * 4) / 4          # heavy ties
    v[2, ::3] = -np.inf                     # masked entries
    v[3, ::5] = np.nan
    v[4] = 0.5                              # all equal
    ld = n + 1 if odd_ld else (n + 3) // 4 * 4
    vt = torch.full((B, ld), -np.inf, device=cuda_device)
    vt[:, :n] = torch.from_numpy(v).to(cuda_device)
    ov = torch.empty((B, segs * k), device=cuda_device)
    oi = torch.empty((B, segs * k), dtype=torch.int64, device=cuda_device)
    L.call("ebt_select_topk", L.ptr(vt), None, ld, B, n, 1000, k, segs, L.ptr(ov), L.ptr(oi),
           segs * k, L.stream_of(cuda_device))
    if segs > 1:
        ov2 = torch.empty((B, k), device=cuda_device)
        oi2 = torch.empty((B, k), dtype=torch.int64, device=cuda_device)
        L.call("ebt_select_topk", L.ptr(ov), L.ptr(oi), segs * k, B, segs * k, 0, k, 1, L.ptr(ov2),
               L.ptr(oi2), k, L.stream_of(cuda_device))
        ov, oi = ov2, oi2
    oi = oi.cpu().numpy()
    ov = ov.cpu().numpy()
    for b in range(B):
        ref = _select_ref(v[b], k)
        got = oi[b]
        m = len(ref)
        np.testing.assert_array_equal(got[:m], ref + 1000)
        np.testing.assert_array_equal(ov[b, :m], v[b][ref])
        assert np.all(got[m:] == -1)


# ----------------------------------------------------------------------- full pipeline ----
@pytest.mark.parametrize("name", sorted(COS_CASES))
def test_cos_topk_golden(cuda_device, name):
    ebt, L = _ebt()
    case = COS_CASES[name]
    q, c, excl = cos_case_inputs(case)
    gold = np.load(os.path.join(GOLD, "cos_topk_small.npz"))
    cat = ebt.Catalog(_t(c, case["dtype"], cuda_device))
    s, r = ebt.score_topk(cat, case["k"], queries=_t(q, case["dtype"], cuda_device),
                          exclude=[list(e) for e in excl] if excl is not None else None)
    assert_topk_equal(s, r, gold[f"{name}_scores"], gold[f"{name}_rows"].astype(np.int64))


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_small_kprime_forces_retry(cuda_device, dt):
    """k' = k leaves no margin: certification must fail and the retry must still be exact."""
    ebt, L = _ebt()
    q = gaussian(2, 200, 256, dt)
    c = gaussian(1, 20000, 256, dt)
    cat = ebt.Catalog(_t(c, dt, cuda_device))
    s, r = ebt.score_topk(cat, 64, queries=_t(q, dt, cuda_device), kprime=64)
    s_ref, r_ref = R.cosine_topk(q, c, 64)
    assert_topk_equal(s, r, s_ref, r_ref)


def test_ties_duplicate_rows(cuda_device):
    """A cluster of 60 identical catalog rows straddles the k boundary: exact ties, resolved
    by row ascending; certification needs a retry with a wider k'."""
    ebt, L = _ebt()
    q = gaussian(2, 8, 64, "f32")
    c = gaussian(1, 5000, 64, "f32")
    dup = np.arange(100, 5000, 80)[:60]
    c[dup] = q[0] * 3.0  # best possible score for query 0, 60 ties
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    s, r = ebt.score_topk(cat, 10, queries=_t(q, "f32", cuda_device))
    s_ref, r_ref = R.cosine_topk(q, c, 10)
    assert_topk_equal(s, r, s_ref, r_ref, atol=1e-12)
    assert list(r[0].cpu().numpy()) == list(dup[:10])


def test_k_larger_than_catalog_and_full_exclusion(cuda_device):
    ebt, L = _ebt()
    q = gaussian(2, 3, 32, "f64")
    c = gaussian(1, 300, 32, "f64")
    cat = ebt.Catalog(_t(c, "f64", cuda_device))
    excl = [list(range(0, 300, 2)), list(range(300)), []]
    s, r = ebt.score_topk(cat, 1000, queries=_t(q, "f64", cuda_device), exclude=excl)
    s_ref, r_ref = R.cosine_topk(q, c, 1000, excl)
    assert_topk_equal(s, r, s_ref, r_ref)
    assert (r[1] == -1).all()


def test_liked_queries_match_oracle(cuda_device):
    ebt, L = _ebt()
    ids, cat_np = c1_catalog()
    cat = ebt.Catalog(_t(cat_np, "f64", cuda_device), ids=ids)
    rng = np.random.default_rng(7)
    liked = [sorted(rng.choice(len(ids), size=int(rng.integers(1, 90)), replace=False).tolist())
             for _ in range(20)]
    liked[0] = [7]  # only the zero-norm row
    excl = [sorted(set(l) | set(rng.choice(len(ids), 30, replace=False).tolist())) for l in liked]
    s, r = ebt.score_topk(cat, 10, liked=liked, exclude=excl)
    s_ref, r_ref = R.liked_topk(cat_np, liked, 10, excl)
    r_np = r.cpu().numpy()
    # row 0 scores are all exactly 0 (zero-norm liked row): tie order = row asc in both
    assert_topk_equal(s, r, s_ref, r_ref)
    assert r_np.shape == (20, 10)


def test_sharded_merge_equals_unsharded(cuda_device):
    ebt, L = _ebt()
    from robot_ebert_amd.distributed import shard_range
    case = COS_CASES["d768_f32_k100"]
    q, c, _ = cos_case_inputs(case)
    qt = _t(q, "f32", cuda_device)
    full = ebt.Catalog(_t(c, "f32", cuda_device))
    s_full, r_full = ebt.score_topk(full, 100, queries=qt)
    parts_s, parts_r = [], []
    for rank in range(5):
        a, b = shard_range(c.shape[0], rank, 5)
        shard = ebt.Catalog(_t(c[a:b], "f32", cuda_device), row_offset=a, n_global=c.shape[0])
        s, r = ebt.score_topk(shard, 100, queries=qt)
        parts_s.append(s)
        parts_r.append(r)
    ms, mr = ebt.merge_topk(torch.stack(parts_s), torch.stack(parts_r), 100)
    assert torch.equal(mr, r_full)
    torch.testing.assert_close(ms, s_full, rtol=0, atol=0)


def test_chunked_catalog_equals_single_chunk(cuda_device):
    ebt, L = _ebt()
    q = gaussian(2, 300, 128, "bf16")
    c = gaussian(1, 50000, 128, "bf16")
    cat = ebt.Catalog(_t(c, "bf16", cuda_device))
    qt = _t(q, "bf16", cuda_device)
    s1, r1 = ebt.score_topk(cat, 50, queries=qt)
    s2, r2 = ebt.score_topk(cat, 50, queries=qt, chunk_rows=4096)
    assert torch.equal(r1, r2)
    s_ref, r_ref = R.cosine_topk(q, c, 50)
    assert_topk_equal(s1, r1, s_ref, r_ref)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_fused_screen_equals_unfused_and_oracle(cuda_device, dt):
    """n >= 2H takes the fused screen (head threshold + GEMM epilogue filter)."""
    ebt, L = _ebt()
    n, d, B, k = 300_000, 256, 300, 40
    c = gaussian(1, n, d, dt)
    q = gaussian(2, B, d, dt)
    rng = np.random.default_rng(3)
    excl = [np.sort(rng.choice(n, 200, replace=False)) for _ in range(B)]
    excl[0] = np.arange(0, n, 3)  # a third of the catalog excluded for query 0
    cat = ebt.Catalog(_t(c, dt, cuda_device))
    qt = _t(q, dt, cuda_device)
    timer = ebt.Timer()
    s1, r1 = ebt.score_topk(cat, k, queries=qt, exclude=[list(e) for e in excl], timer=timer)
    assert timer.query("gemm_filter")[1] >= 1, "fused path not taken"
    s2, r2 = ebt.score_topk(cat, k, queries=qt, exclude=[list(e) for e in excl], fuse=False)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(s1, s2, rtol=0, atol=0)
    sample = list(range(0, B, 25))
    s_ref, r_ref = R.cosine_topk(q[sample], c, k, [excl[i] for i in sample])
    assert_topk_equal(s1[sample], r1[sample], s_ref, r_ref)


@pytest.mark.parametrize("B", [100, 300])
def test_fused_large_kprime_block_path(cuda_device, B):
    """k' > 512 (C5's k = 1000 class) with block-level merges: B = 100 (B_pad 128, no sample)
    takes the 256 k'-row head; B = 300 the speculative screen (sample threshold). Both equal
    the unfused path and the oracle on sampled queries, with exclusions."""
    ebt, L = _ebt()
    n, d, k = 400_000, 128, 600
    c = gaussian(4, n, d, "f16")
    q = gaussian(5, B, d, "f16")
    rng = np.random.default_rng(6)
    excl = [np.sort(rng.choice(n, 500, replace=False)) for _ in range(B)]
    cat = ebt.Catalog(_t(c, "f16", cuda_device))
    qt = _t(q, "f16", cuda_device)
    pl = ebt.search.plan(cat, B, k)
    assert pl["fused"] and pl["kprime"] > 512
    if B <= 128:
        assert pl["spec"] is None and pl["head_rows"] >= 256 * pl["kprime"], pl
    else:
        assert pl["spec"] is not None, pl
    timer = ebt.Timer()
    s1, r1 = ebt.score_topk(cat, k, queries=qt, exclude=[list(e) for e in excl], timer=timer)
    assert timer.query("gemm_filter")[1] >= 1, "fused path not taken"
    s2, r2 = ebt.score_topk(cat, k, queries=qt, exclude=[list(e) for e in excl], fuse=False)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(s1, s2, rtol=0, atol=0)
    sample = [0, 64, B - 1]
    s_ref, r_ref = R.cosine_topk(q[sample].astype(np.float64), c.astype(np.float64), k,
                                 [excl[i] for i in sample])
    assert_topk_equal(s1[sample], r1[sample], s_ref, r_ref)


def test_block_merge_deferred_tier(cuda_device, monkeypatch):
    """The block merge's two tiers: EBT_MERGE_MARGIN=0 sizes the first (small-LDS) pass for
    k' + 256 entries, so queries with more hits are deferred to the full-size pass; the answer
    is the same as the unfused path's."""
    ebt, L = _ebt()
    n, d, k, B = 400_000, 128, 600, 300
    c = gaussian(4, n, d, "f16")
    q = gaussian(5, B, d, "f16")
    cat = ebt.Catalog(_t(c, "f16", cuda_device))
    qt = _t(q, "f16", cuda_device)
    assert ebt.search.plan(cat, B, k)["spec"] is not None
    s2, r2 = ebt.score_topk(cat, k, queries=qt, fuse=False)
    for margin in ("0", "3"):
        monkeypatch.setenv("EBT_MERGE_MARGIN", margin)
        s1, r1 = ebt.score_topk(cat, k, queries=qt)
        assert torch.equal(r1, r2), margin
        torch.testing.assert_close(s1, s2, rtol=0, atol=0)


def test_speculative_screen_matches_oracle(cuda_device):
    """The speculative fused screen (pooled sample threshold, one filter pass, verify) on a
    shape where it is the default: bit-exact rows vs the oracle, equal to the unfused path."""
    ebt, L = _ebt()
    n, d, B, k = 98_304, 96, 300, 20
    c = gaussian(21, n, d, "f32")
    q = gaussian(22, B, d, "f32")
    rng = np.random.default_rng(23)
    excl = [np.sort(rng.choice(n, 40, replace=False)) for _ in range(B)]
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    qt = _t(q, "f32", cuda_device)
    pl = ebt.search.plan(cat, B, k)
    assert pl["fused"] and pl["spec"] is not None and pl["spec"]["tiles"] >= 8, pl
    timer = ebt.Timer()
    s1, r1 = ebt.score_topk(cat, k, queries=qt, exclude=[list(e) for e in excl], timer=timer)
    assert timer.query("gemm_filter")[1] >= 1
    s2, r2 = ebt.score_topk(cat, k, queries=qt, exclude=[list(e) for e in excl], fuse=False)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(s1, s2, rtol=0, atol=0)
    s_ref, r_ref = R.cosine_topk(q.astype(np.float64), c.astype(np.float64), k,
                                 [list(e) for e in excl])
    assert_topk_equal(s1, r1, s_ref, r_ref)


def test_speculative_threshold_failure_reruns(cuda_device):
    """Near-duplicates of query 0 placed only in the SAMPLE tiles make its speculative
    threshold (the sample's j-th best) exceed T - 2 eps: the verify step flags it (ovf = 2, cert
    -1), the query is rerun unfused, and the result is still exact."""
    ebt, L = _ebt()
    from robot_ebert_amd.search import prepare_queries, run_screen
    n, d, B, k = 98_304, 64, 256, 10
    c = gaussian(31, n, d, "f32")
    q = gaussian(32, B, d, "f32")
    cat0 = ebt.Catalog(_t(c, "f32", cuda_device))
    sp = ebt.search.plan(cat0, B, k)["spec"]
    assert sp is not None
    rng = np.random.default_rng(33)
    lead = sp.get("lead", 0)
    for t in range(sp["tiles"]):   # the sample: tiles 0 .. lead-1, then every stride-th from lead
        row0 = 256 * (t if t < lead else lead + (t - lead) * sp["stride"])
        for r in range(4):  # 4 near-duplicates per sample tile: >> the rank j in the sample
            c[row0 + 17 * r] = q[0] + 1e-3 * rng.standard_normal(d)
    c = c.astype(np.float32)  # the oracle sees the values the GPU catalog holds
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    qt = _t(q, "f32", cuda_device)
    qb = prepare_queries(cat, queries=qt)
    kp = ebt.search.plan(cat, B, k)["kprime"]
    lv, lr, ovf, eps = run_screen(cat, qb, k, kp)
    assert int(ovf[0]) == 2, "the verify step did not catch the bad speculative threshold"
    s, r = ebt.score_topk(cat, k, queries=qt)
    sample = [0, 1, 100, 255]
    s_ref, r_ref = R.cosine_topk(q[sample].astype(np.float64), c.astype(np.float64), k)
    assert_topk_equal(s[sample], r[sample], s_ref, r_ref)


def test_submit_finish_pipelined_equals_sync(cuda_device):
    """score_topk_submit of batch i+1 before score_topk_finish of batch i (bench.py's step
    loop): each batch's result equals its synchronous score_topk, including a batch whose
    queries need retries (near-duplicates: certificate 0 -> widened k')."""
    ebt, L = _ebt()
    n, d, k = 70_000, 64, 16
    c = gaussian(41, n, d, "f32")
    qa = gaussian(42, 300, d, "f32")
    qb = gaussian(43, 300, d, "f32")
    c[1000:1400] = (qb[0] + 1e-7 * np.arange(400)[:, None]).astype(np.float32)  # a near-tie wall
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    ta, tb = _t(qa, "f32", cuda_device), _t(qb, "f32", cuda_device)
    pa = ebt.score_topk_submit(cat, k, queries=ta)
    pb = ebt.score_topk_submit(cat, k, queries=tb)
    sa, ra = ebt.score_topk_finish(pa)
    sb, rb = ebt.score_topk_finish(pb)
    for (s, r, t) in ((sa, ra, ta), (sb, rb, tb)):
        s2, r2 = ebt.score_topk(cat, k, queries=t)
        assert torch.equal(r, r2)
        torch.testing.assert_close(s, s2, rtol=0, atol=0)
    s_ref, r_ref = R.cosine_topk(qb[:4].astype(np.float64), c.astype(np.float64), k)
    assert_topk_equal(sb[:4], rb[:4], s_ref, r_ref)


def test_fused_overflow_falls_back(cuda_device):
    """Scores that grow with the row index make the head threshold useless: every tail row
    passes, the candidate list overflows, and the query must be redone unfused -- exactly."""
    ebt, L = _ebt()
    n, d, k = 200_000, 64, 16
    rng = np.random.default_rng(9)
    q = rng.standard_normal((2, d))
    t = (np.arange(n) / n)[:, None]
    c = q[0][None, :] * t + rng.standard_normal((n, d)) * (1.0 - t) * 0.5
    cat = ebt.Catalog(_t(c, "f64", cuda_device))
    s, r = ebt.score_topk(cat, k, queries=_t(q, "f64", cuda_device))
    s_ref, r_ref = R.cosine_topk(q, c, k)
    assert_topk_equal(s, r, s_ref, r_ref)


# ----------------------------------------------------------- the reference call surface ----
def _collab_setup(cuda_device):
    ebt, L = _ebt()
    from sqlalchemy import create_engine, insert
    from robot_ebert_amd import lib, tables
    from robot_ebert_amd.models import Movie
    with open(os.path.join(GOLD, "c1_collab.json")) as f:
        gold = json.load(f)
    ids, cat_np = c1_catalog()
    from sqlalchemy.pool import StaticPool
    # one in-memory database shared by every thread (the batched test runs 16 request threads)
    engine = create_engine("sqlite://", connect_args={"check_same_thread": False},
                           poolclass=StaticPool)
    tables.ratings.create(engine)
    with engine.begin() as cnx:
        for uid, rec in gold["users"].items():
            for t, rt in rec["ratings"]:
                cnx.execute(insert(tables.ratings).values(user_id=uid, tmdb_id=t, rating=rt))
    pop = dict(zip(gold["search"]["match_ids"], gold["search"]["popularity"]))

    def movies(tmdb_ids):
        import datetime
        return [Movie(tmdb_id=t, tmdb_homepage="", title=t, language="en",
                      release_date=datetime.date(2000, 1, 1), runtime=90, director="d",
                      actors=None, genres=None, keywords=None, overview="", budget=0, revenue=0,
                      popularity=pop.get(t, 1.0), vote_average=0.0, vote_count=0)
                for t in sorted(tmdb_ids)]

    lib.configure(engine=engine, catalog=ebt.Catalog(_t(cat_np, "f64", cuda_device), ids=ids),
                  get_movies=movies)
    return lib, gold


@pytest.mark.parametrize("k", [10, 10000])
def test_get_user_recs_matches_reference(cuda_device, k):
    lib, gold = _collab_setup(cuda_device)
    for uid, rec in gold["users"].items():
        want = rec[f"k{k}"]
        if isinstance(want, dict):
            with pytest.raises(ValueError) as ei:
                lib.get_user_recs(uid, k)
            assert str(ei.value) == want["message"]
            continue
        got = lib.get_user_recs(uid, k)
        assert [g.movie.tmdb_id for g in got] == [w[0] for w in want], uid
        np.testing.assert_allclose([g.score for g in got], [w[1] for w in want], rtol=0,
                                   atol=SCORE_ATOL)


def test_search_rerank_matches_reference(cuda_device):
    lib, gold = _collab_setup(cuda_device)
    s = gold["search"]
    for uid, want in s["cases"].items():
        user = None if uid == "None" else uid
        if isinstance(want, dict):
            with pytest.raises(ValueError):
                lib.rerank_search_matches(s["match_ids"], s["match_scores"], user)
            continue
        got = lib.rerank_search_matches(s["match_ids"], s["match_scores"], user)
        assert [g.movie.tmdb_id for g in got] == [w[0] for w in want]
        np.testing.assert_allclose([g.score for g in got], [w[1] for w in want], atol=1e-12)


@pytest.mark.parametrize("k", [10, 10000])
def test_batched_user_recs_match_reference(cuda_device, k):
    """§8f-2: 16 request threads through one RecBatcher give get_user_recs' golden answers
    (errors per request, ordering), and the GPU saw coalesced batches."""
    import concurrent.futures as cf
    from robot_ebert_amd.batcher import RecBatcher
    lib, gold = _collab_setup(cuda_device)
    b = RecBatcher(lib.movies_collab_catalog, max_batch=64, max_wait_ms=20.0)
    users = list(gold["users"].items())

    def one(item):
        uid, rec = item
        try:
            return uid, rec, lib.get_user_recs_batched(b, uid, k), None
        except ValueError as e:
            return uid, rec, None, e
    with cf.ThreadPoolExecutor(16) as ex:
        out = list(ex.map(one, users))
    b.close()
    for uid, rec, got, err in out:
        want = rec[f"k{k}"]
        if isinstance(want, dict):
            assert err is not None and str(err) == want["message"], uid
            continue
        assert err is None, (uid, err)
        assert [g.movie.tmdb_id for g in got] == [w[0] for w in want], uid
        np.testing.assert_allclose([g.score for g in got], [w[1] for w in want], rtol=0,
                                   atol=SCORE_ATOL)
    assert max(b.batches) > 1


def test_score_server_user_recs_match_reference(cuda_device):
    """§8f-2, the multi-process shape (serving.py): the route's requests go through ScoreClients
    (three connections, as three server processes would hold) to one ScoreServer over the GPU
    RecBatcher; the answers are get_user_recs' golden ones at k = 10, errors keep their text,
    and the server coalesced requests of different connections into one batch."""
    import concurrent.futures as cf
    from robot_ebert_amd.batcher import RecBatcher
    from robot_ebert_amd.serving import ScoreClient, ScoreServer
    lib, gold = _collab_setup(cuda_device)
    b = RecBatcher(lib.movies_collab_catalog, max_batch=64, max_wait_ms=20.0)
    srv = ScoreServer(b)
    clients = [ScoreClient(srv.address) for _ in range(3)]
    users = list(gold["users"].items())

    def one(i):
        uid, rec = users[i]
        try:
            return uid, rec, lib.get_user_recs_batched(clients[i % 3], uid, 10), None
        except ValueError as e:
            return uid, rec, None, e
    try:
        with cf.ThreadPoolExecutor(16) as ex:
            out = list(ex.map(one, range(len(users))))
    finally:
        for c in clients:
            c.close()
        srv.close()
        b.close()
    for uid, rec, got, err in out:
        want = rec["k10"]
        if isinstance(want, dict):
            assert err is not None and str(err) == want["message"], uid
            continue
        assert err is None, (uid, err)
        assert [g.movie.tmdb_id for g in got] == [w[0] for w in want], uid
        np.testing.assert_allclose([g.score for g in got], [w[1] for w in want], rtol=0,
                                   atol=SCORE_ATOL)
    assert srv.requests > 0 and max(b.batches) > 1


def test_catalog_from_chroma_matches_reference(cuda_device):
    """§8f-3: the C1 catalog ingested from a Chroma-style get() result (ids + embeddings, the
    constants.py:55-56 source) serves get_user_recs with the reference's golden answers."""
    from robot_ebert_amd import ingest
    lib, gold = _collab_setup(cuda_device)
    ids, cat_np = c1_catalog()
    cat = ingest.catalog_from_chroma({"ids": ids, "embeddings": cat_np.tolist()}, device=cuda_device)
    lib.configure(catalog=cat, get_movies=lib._get_movies_override)
    for uid, rec in list(gold["users"].items())[:8]:
        want = rec["k10"]
        if isinstance(want, dict):
            continue
        got = lib.get_user_recs(uid, 10)
        assert [g.movie.tmdb_id for g in got] == [w[0] for w in want], uid


def test_exact_content_search(cuda_device):
    """§8f-1: run_search's retrieval as exact cosine top-k over a 1536-d content catalog (HNSW
    parity unpinned: compared with the float64 oracle), then the reference re-ranking."""
    from robot_ebert_amd import lib as L_
    lib, gold = _collab_setup(cuda_device)
    ids, _ = c1_catalog()
    rng = np.random.default_rng(77)
    content = rng.standard_normal((len(ids), 1536))
    lib.configure(content_catalog=ebt_catalog(content, ids, cuda_device),
                  get_movies=lib._get_movies_override)
    qe = rng.standard_normal(1536)
    got_ids, got_s = lib.retrieve_content_matches(qe, 10)
    s_ref, r_ref = R.cosine_topk(qe[None, :], content, 10)
    assert got_ids == [ids[i] for i in r_ref[0]]
    np.testing.assert_allclose(got_s, s_ref[0], rtol=0, atol=SCORE_ATOL)
    recs = lib.run_search_exact(qe, None, 10)
    want = lib.rerank_search_matches(got_ids, got_s, None)
    assert [r.movie.tmdb_id for r in recs] == [w.movie.tmdb_id for w in want]


def ebt_catalog(x, ids, dev):
    ebt, _ = _ebt()
    return ebt.Catalog(_t(x, "f64", dev), ids=ids)


# ------------------------------------------------------------------ full-size properties ----
def test_c3_shape_sample_parity(cuda_device):
    """Headline shape class (d=1536 f32) at 200K rows: sampled queries vs the oracle."""
    ebt, L = _ebt()
    n, d, B, k = 200_000, 1536, 512, 100
    g = torch.Generator(device=cuda_device).manual_seed(1)
    c = torch.randn((n, d), generator=g, device=cuda_device)
    q = torch.randn((B, d), generator=torch.Generator(device=cuda_device).manual_seed(2),
                    device=cuda_device)
    cat = ebt.Catalog(c)
    s, r = ebt.score_topk(cat, k, queries=q)
    sample = np.arange(0, B, 32)
    s_ref, r_ref = R.cosine_topk(q[sample].cpu().numpy(), c.cpu().numpy(), k)
    assert_topk_equal(s[sample], r[sample], s_ref, r_ref)
    # properties on every query: sorted, unique rows, scores in [-1, 1]
    sn = s.cpu().numpy()
    assert np.all(np.diff(sn, axis=1) <= 0)
    assert np.all(np.abs(sn) <= 1 + 1e-12)
    rn = r.cpu().numpy()
    assert all(len(set(x)) == k for x in rn)


# ------------------------------------------------------------------ torch custom ops ----
@pytest.mark.parametrize("case", ["d768_f32_k100_excl", "d1536_bf16_k10", "d200_f64_k50"])
def test_torch_ops_cosine_topk(cuda_device, case):
    """torch.ops.ebert.{row_norms, screen_image, cosine_topk, merge_topk} on plain tensors vs
    the float64 oracle (golden case inputs, exclusions), and a 2-shard merge through the op."""
    ebt, L = _ebt()
    c = COS_CASES[case]
    qv, cat_np, excl = cos_case_inputs(c)
    k = c["k"]
    cat = _t(cat_np, c["dtype"], cuda_device)
    q = _t(qv, c["dtype"], cuda_device)
    g, inv = torch.ops.ebert.row_norms(cat)
    img = torch.ops.ebert.screen_image(cat, g)
    eo = er = None
    if excl is not None:
        eo = torch.tensor(np.concatenate([[0], np.cumsum([len(e) for e in excl])]),
                          dtype=torch.int64, device=cuda_device)
        er = torch.tensor(np.concatenate([np.sort(e) for e in excl]), dtype=torch.int64,
                          device=cuda_device)
    s, r = torch.ops.ebert.cosine_topk(q, cat, g, inv, img, k, eo, er, 0)
    s_ref, r_ref = R.cosine_topk(qv.astype(np.float64), cat_np.astype(np.float64), k, excl)
    assert_topk_equal(s, r, s_ref, r_ref)
    # two shards + merge through the op
    h = cat.shape[0] // 2
    parts = []
    for a, b in ((0, h), (h, cat.shape[0])):
        gs, invs = torch.ops.ebert.row_norms(cat[a:b])
        ims = torch.ops.ebert.screen_image(cat[a:b], gs)
        parts.append(torch.ops.ebert.cosine_topk(q, cat[a:b], gs, invs, ims, k, eo, er, a))
    ms, mr = torch.ops.ebert.merge_topk(torch.stack([p[0] for p in parts]),
                                        torch.stack([p[1] for p in parts]), k)
    assert_topk_equal(ms, mr, s_ref, r_ref)


@pytest.mark.parametrize("qdt,cdt,d", [("f32", "f32", 1536), ("bf16", "bf16", 768),
                                       ("f16", "f16", 200), ("f64", "f64", 32),
                                       ("f16", "f32", 4096)])
def test_query_prep_fused_equals_two_kernels(cuda_device, qdt, cdt, d):
    """ebt_query_prep (one launch) writes what ebt_query_dense + ebt_query_image write, native
    images included: bitwise for the block-per-query form (d = 4096 here); the wave-per-query
    form (16-byte rows, d % 8 == 0, d <= 2048) sums the norms in another order, so q64 within
    4 ulp, the image bitwise except where that moves a value across an f16/bf16 rounding
    boundary (then one unit), scale and eps within float32 rounding."""
    ebt, L = _ebt()
    from robot_ebert_amd.search import pad_batch
    B = 300
    cat = ebt.Catalog(_t(gaussian(41, 1000, d, cdt), cdt, cuda_device))
    q = _t(gaussian(42, B, d, qdt), qdt, cuda_device)
    qb = ebt.prepare_queries(cat, queries=q)          # the fused launch (d <= 4096)
    st = L.stream_of(cuda_device)
    q64 = torch.empty((B, d), dtype=torch.float64, device=cuda_device)
    L.call("ebt_query_dense", L.ptr(q), L.DTYPE_CODE[q.dtype], B, d, d, L.ptr(q64), st)
    B_pad = pad_batch(B)
    native = cat.native and q.dtype == cat.img_torch_dtype
    qimg = torch.empty((B_pad, cat.ld_img), dtype=cat.img_torch_dtype, device=cuda_device)
    qs = torch.empty(B_pad, dtype=torch.float32, device=cuda_device)
    eps = torch.empty(B_pad, dtype=torch.float32, device=cuda_device)
    L.call("ebt_query_image", L.ptr(q64), B, B_pad, d, cat.img_dtype, L.ptr(q) if native else None,
           d if native else 0, 1 if native else 0, float(cat.u_cat), L.ptr(qimg), cat.ld_img,
           L.ptr(qs), L.ptr(eps), st)
    if d > 2048:
        assert torch.equal(qb.q64, q64)
        assert torch.equal(qb.qimg.view(torch.int16), qimg.view(torch.int16))
        assert torch.equal(qb.qscale, qs) and torch.equal(qb.eps, eps)
        return
    assert torch.allclose(qb.q64, q64, rtol=4 * 2.0 ** -52, atol=0)
    a, b = qb.qimg.view(torch.int16).int(), qimg.view(torch.int16).int()
    assert int((a - b).abs().max()) <= 1
    assert float((a == b).double().mean()) >= 0.999
    assert torch.allclose(qb.qscale, qs, rtol=2.0 ** -22, atol=0)
    assert torch.allclose(qb.eps, eps, rtol=2.0 ** -22, atol=0)


@pytest.mark.parametrize("eps_v", [0.0, 0.002, 0.05])
def test_rescore_two_stage_cut(cuda_device, eps_v):
    """ebt_rescore's raised cut (s_min - eps, s_min = the smallest exact score of the list's
    first k): approx values perturbed within +-eps of the exact scores, the list = the k' best
    approx of the whole catalog. Its top k equals the exact top k of the candidates; with
    certified = 1 it is the catalog's exact top k; eps = 0 with equal cand_vals rescores every
    candidate (the header's contract)."""
    ebt, L = _ebt()
    n, d, B, k, kp = 3000, 48, 6, 20, 300
    rng = np.random.default_rng(7)
    cat = rng.standard_normal((n, d))
    q = rng.standard_normal((B, d))
    q64 = q / np.linalg.norm(q, axis=1, keepdims=True)
    g = np.linalg.norm(cat, axis=1)
    exact = (q64 @ cat.T) / g
    if eps_v > 0:
        approx = (exact + rng.uniform(-0.9 * eps_v, 0.9 * eps_v, exact.shape)).astype(np.float32)
    else:
        approx = exact.astype(np.float32)
    cand = np.argsort(-approx.astype(np.float64), axis=1, kind="stable")[:, :kp]
    cv = np.take_along_axis(approx, cand, 1)
    if eps_v == 0.0:
        cv[:] = 0.0  # the "rescore every candidate" form
    dev = cuda_device
    T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x)).to(dev).to(dt)
    qt, ct, gt = T(q64, torch.float64), T(cat, torch.float64), T(g, torch.float64)
    cvt, crt = T(cv, torch.float32), T(cand, torch.int64)
    epst = torch.full((B,), eps_v, dtype=torch.float32, device=dev)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    cert = torch.empty(B, dtype=torch.int32, device=dev)
    L.call("ebt_rescore", L.ptr(qt), B, d, L.ptr(ct), L.DTYPE_CODE[torch.float64], d, L.ptr(gt),
           0, L.ptr(cvt), L.ptr(crt), kp, k, n, L.ptr(epst), None, L.ptr(out_s), L.ptr(out_r),
           L.ptr(cert), None, L.stream_of(dev))
    torch.cuda.synchronize()
    s, r, c = out_s.cpu().numpy(), out_r.cpu().numpy(), cert.cpu().numpy()
    for b in range(B):
        ce = exact[b, cand[b]]
        o = np.lexsort((cand[b], -ce))[:k]
        np.testing.assert_array_equal(r[b], cand[b][o])
        np.testing.assert_allclose(s[b], ce[o], rtol=0, atol=SCORE_ATOL)
        if c[b] == 1:
            np.testing.assert_array_equal(r[b], np.lexsort((np.arange(n), -exact[b]))[:k])
    if eps_v == 0.002:
        assert (c == 1).all()


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_unsorted_device_exclusions(cuda_device, dt):
    """A caller's device CSR with UNSORTED segments: the fused merge binary-searches
    exclusions, so score_topk / torch.ops.ebert.cosine_topk must sort them first. The excluded
    rows are drawn from each query's true top 200, so keeping any of them changes the answer."""
    ebt, L = _ebt()
    from robot_ebert_amd.search import plan
    n, d, B, k = 65536, 256, 256, 100
    c = gaussian(31, n, d, dt)
    qv = gaussian(32, B, d, dt)
    s0, r0 = R.cosine_topk(qv, c, 200)
    rng = np.random.default_rng(33)
    excl = [rng.permutation(np.concatenate([r0[b, rng.choice(200, 60, replace=False)],
                                            rng.choice(n, 40, replace=False)]))
            for b in range(B)]
    excl = [np.array(list(dict.fromkeys(e.tolist())), dtype=np.int64) for e in excl]  # unique
    eo = torch.tensor(np.concatenate([[0], np.cumsum([len(e) for e in excl])]),
                      dtype=torch.int64, device=cuda_device)
    er = torch.tensor(np.concatenate(excl), dtype=torch.int64, device=cuda_device)
    assert any(np.any(np.diff(e) < 0) for e in excl)
    cat = ebt.Catalog(_t(c, dt, cuda_device))
    assert plan(cat, B, k)["fused"]
    q = _t(qv, dt, cuda_device)
    s_ref, r_ref = R.cosine_topk(qv, c, k, excl)
    s, r = ebt.score_topk(cat, k, queries=q, exclude=(eo, er))
    assert_topk_equal(s, r, s_ref, r_ref)
    g, inv = torch.ops.ebert.row_norms(cat.data)
    img = torch.ops.ebert.screen_image(cat.data, g)
    s2, r2 = torch.ops.ebert.cosine_topk(q, cat.data, g, inv, img, k, eo, er, 0)
    assert_topk_equal(s2, r2, s_ref, r_ref)


@pytest.mark.parametrize("dt,d,ld,img", [("f32", 1536, 1536, 2), ("f32", 77, 80, 2),
                                          ("f64", 200, 200, 1), ("bf16", 72, 72, 2),
                                          ("f16", 130, 136, 1), ("f32", 77, 77, 1)])
def test_screen_image_bitwise(cuda_device, dt, d, ld, img):
    """ebt_screen_image (one wave per row, 16-byte vector loads where the rows allow it, the
    element form for a ragged last chunk or an unaligned stride): round_to(img, x * (1/gnorm))
    in float64 -> float32 -> f16/bf16 within the certificate's rounding bound and bitwise equal
    to torch's conversion but for rare ties, zero columns past d."""
    ebt, L = _ebt()
    n = 1000
    x = torch.randn((n, ld), generator=torch.Generator().manual_seed(d), dtype=torch.float64)
    x[3] = 0.0                                          # the zero-norm guard
    xt = x.to(TORCH_DT[dt]).to(cuda_device)
    g = torch.empty(n, dtype=torch.float64, device=cuda_device)
    L.call("ebt_row_norms", L.ptr(xt), L.DTYPE_CODE[xt.dtype], n, d, ld, L.ptr(g), None,
           L.stream_of(cuda_device))
    ld_img = (d + 63) // 64 * 64
    out = torch.full((n, ld_img), 7, dtype=torch.int16, device=cuda_device)
    for normalize in (1, 0):
        L.call("ebt_screen_image", L.ptr(xt), L.DTYPE_CODE[xt.dtype], n, d, ld, L.ptr(g),
               normalize, img, L.ptr(out), ld_img, L.stream_of(cuda_device))
        xd = xt[:, :d].double()
        s = (1.0 / g) if normalize else torch.ones_like(g)
        want = (xd * s[:, None]).float().to(torch.float16 if img == 2 else torch.bfloat16)
        got = out[:, :d].view(torch.float16 if img == 2 else torch.bfloat16)
        # the device's double rounding (f64 -> f32 -> 16-bit) can land on the other side of a
        # 16-bit tie than torch's in rare cases (a few per 10^5 elements): the certificate
        # (prep.hip) needs |img - x/|x|| <= 1.05 u |x/|x||, u = 2^-11
        # (f16) / 2^-8 (bf16), plus the f16 subnormal spacing
        v = xd * s[:, None]
        u = 2.0 ** -11 if img == 2 else 2.0 ** -8
        err = (got.double() - v).abs()
        assert bool((err <= 1.01 * u * v.abs() + 2.0 ** -25).all()), float((err / v.abs()).max())
        same = (got.view(torch.int16) == want.view(torch.int16)).double().mean().item()
        assert same >= 0.9999, same
        assert bool((out[:, d:] == 0).all())


def test_exclusion_csr_with_offset_start(cuda_device):
    """a device CSR whose offsets start past 0 (a sub-batch slicing the offsets of a
    larger CSR), with unsorted segments and foreign rows before off[0] and after off[-1]: the
    library's segmented sort (ebt_sort_exclusions) sorts each segment in place by its ABSOLUTE
    positions and leaves the rest alone, so every query excludes exactly its own rows."""
    ebt, L = _ebt()
    from robot_ebert_amd.search import csr_sorted
    n, d, B, k = 40_000, 128, 256, 50
    c = gaussian(35, n, d, "f32")
    qv = gaussian(36, B, d, "f32")
    s0, r0 = R.cosine_topk(qv, c, 120)
    rng = np.random.default_rng(37)
    excl = [rng.permutation(np.unique(np.concatenate([r0[b, rng.choice(120, 30, replace=False)],
                                                      rng.choice(n, 20, replace=False)])))
            for b in range(B)]
    excl[5] = np.array([], dtype=np.int64)              # an empty segment
    junk_head = r0[:7, 0]                               # top rows of other queries
    junk_tail = r0[7:12, 0]
    flat = np.concatenate([junk_head] + excl + [junk_tail]).astype(np.int64)
    off = np.concatenate([[0], np.cumsum([len(e) for e in excl])]) + len(junk_head)
    eo = torch.tensor(off, dtype=torch.int64, device=cuda_device)
    er = torch.tensor(flat, dtype=torch.int64, device=cuda_device)
    so, sr = csr_sorted(eo, er)
    got = sr.cpu().numpy()
    assert np.array_equal(got[:len(junk_head)], junk_head)
    assert np.array_equal(got[off[-1]:], junk_tail)
    for b in range(B):
        assert np.array_equal(got[off[b]:off[b + 1]], np.sort(excl[b]))
    assert torch.equal(er.cpu(), torch.tensor(flat))    # the caller's CSR is not modified
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    q = _t(qv, "f32", cuda_device)
    s_ref, r_ref = R.cosine_topk(qv, c, k, excl)
    s, r = ebt.score_topk(cat, k, queries=q, exclude=(eo, er))
    assert_topk_equal(s, r, s_ref, r_ref)


def test_sort_exclusions_entry(cuda_device):
    """ebt_sort_exclusions through bare ctypes: in place (rows_out == rows_in), long segments
    (beyond one workgroup), malformed offsets clamped (never read out of bounds)."""
    ebt, L = _ebt()
    rng = np.random.default_rng(38)
    lens = [0, 1, 7, 5000, 300, 0, 70_000, 2]
    rows = [rng.integers(-5, 1 << 40, size=m) for m in lens]
    off = np.concatenate([[0], np.cumsum(lens)])
    flat = np.concatenate(rows).astype(np.int64)
    eo = torch.tensor(off, dtype=torch.int64, device=cuda_device)
    er = torch.tensor(flat, dtype=torch.int64, device=cuda_device)
    B, nnz = len(lens), len(flat)
    need = L.load().ebt_sort_exclusions_bytes(B, nnz)
    assert need > 0
    ws = torch.empty(need, dtype=torch.uint8, device=cuda_device)
    L.call("ebt_sort_exclusions", L.ptr(eo), L.ptr(er), L.ptr(er), B, nnz, L.ptr(ws), need,
           L.stream_of(cuda_device))
    got = er.cpu().numpy()
    for b in range(B):
        assert np.array_equal(got[off[b]:off[b + 1]], np.sort(rows[b]))
    # offsets past nnz / decreasing: clamped into [0, nnz], the call succeeds and stays in
    # bounds (what the overlapping clamped segments hold afterwards is unspecified); the search
    # entry then rejects the malformed CSR itself
    bad = torch.tensor([0, 10, 5, nnz + 100], dtype=torch.int64, device=cuda_device)
    er2 = torch.tensor(flat, dtype=torch.int64, device=cuda_device)
    need3 = L.load().ebt_sort_exclusions_bytes(3, nnz)
    ws3 = torch.empty(need3, dtype=torch.uint8, device=cuda_device)
    L.call("ebt_sort_exclusions", L.ptr(bad), L.ptr(er2), L.ptr(er2), 3, nnz, L.ptr(ws3), need3,
           L.stream_of(cuda_device))
    torch.cuda.synchronize(cuda_device)
    # (in bounds, but segment 1 runs backwards: every kernel reads an empty range there)
    bad2 = torch.tensor([0, 10, 5, nnz], dtype=torch.int64, device=cuda_device)
    cat = ebt.Catalog(torch.randn((5000, 64), device=cuda_device))
    with pytest.raises(L.EbertError):
        ebt.score_topk(cat, 10, queries=torch.randn((3, 64), device=cuda_device),
                       exclude=(bad2, torch.zeros(nnz, dtype=torch.int64, device=cuda_device)))
    with pytest.raises(L.EbertError):
        L.call("ebt_sort_exclusions", L.ptr(eo), L.ptr(er), L.ptr(er), B, nnz, L.ptr(ws), 16,
               L.stream_of(cuda_device))


def test_sort_exclusions_out_of_place_head_tail(cuda_device):
    """out of place, with off[0] > 0, off[B] < nnz and a decreasing offset, the rows
    outside every clamped segment are copied from rows_in (the sort's copy blocks), the
    well-formed segments come out sorted, and rows_in is not modified. Also: segments beyond one
    LDS run (4096 rows) out of place, sorted and already-sorted (copied)."""
    ebt, L = _ebt()
    rng = np.random.default_rng(39)
    nnz = 30_000
    flat = rng.integers(-1000, 1 << 40, size=nnz).astype(np.int64)
    # segments: [100, 600) [600, 5000) [5000, 5000) [4000, 9000) (overlaps: off decreases)
    # [9000, 9000) ... [9000, 20000) (long, sorted); tail [20000, 30000) untouched
    flat[9000:20000] = np.sort(flat[9000:20000])
    off = np.array([100, 600, 5000, 4000, 9000, 9000, 20000], dtype=np.int64)
    B = len(off) - 1
    er = torch.tensor(flat, device=cuda_device)
    eo = torch.tensor(off, device=cuda_device)
    out = torch.full_like(er, 7)
    need = L.load().ebt_sort_exclusions_bytes(B, nnz)
    ws = torch.empty(need, dtype=torch.uint8, device=cuda_device)
    L.call("ebt_sort_exclusions", L.ptr(eo), L.ptr(er), L.ptr(out), B, nnz, L.ptr(ws), need,
           L.stream_of(cuda_device))
    got = out.cpu().numpy()
    assert np.array_equal(er.cpu().numpy(), flat)           # the input is not modified
    assert np.array_equal(got[:100], flat[:100])            # head
    assert np.array_equal(got[20000:], flat[20000:])        # tail
    assert np.array_equal(got[100:600], np.sort(flat[100:600]))
    assert np.array_equal(got[9000:20000], flat[9000:20000])  # already sorted: copied
    # a long unsorted segment out of place, then in place: both sorted, same result
    off2 = np.array([5, 25_000], dtype=np.int64)
    eo2 = torch.tensor(off2, device=cuda_device)
    out2 = torch.full_like(er, 7)
    need2 = L.load().ebt_sort_exclusions_bytes(1, nnz)
    ws2 = torch.empty(need2, dtype=torch.uint8, device=cuda_device)
    L.call("ebt_sort_exclusions", L.ptr(eo2), L.ptr(er), L.ptr(out2), 1, nnz, L.ptr(ws2), need2,
           L.stream_of(cuda_device))
    g2 = out2.cpu().numpy()
    assert np.array_equal(g2[:5], flat[:5]) and np.array_equal(g2[25_000:], flat[25_000:])
    assert np.array_equal(g2[5:25_000], np.sort(flat[5:25_000]))
    er3 = er.clone()
    L.call("ebt_sort_exclusions", L.ptr(eo2), L.ptr(er3), L.ptr(er3), 1, nnz, L.ptr(ws2), need2,
           L.stream_of(cuda_device))
    assert np.array_equal(er3.cpu().numpy(), g2)


def test_unsorted_exclusions_rejected_by_the_rescore_check(cuda_device):
    """Round 6: the C entry's exclusion-order check is folded into the rescore (certificate -3
    for a query whose segment is not ascending): an unsorted device CSR handed straight to
    ebt_cosine_topk fails with the same message; the same CSR sorted passes; a SortedCSR from
    csr_sorted / csr_from_lists is used as it is."""
    ebt, L = _ebt()
    from robot_ebert_amd.search import SortedCSR, csr_from_lists, csr_sorted
    n, d, B, k = 20_000, 64, 300, 10
    cat = ebt.Catalog(torch.randn((n, d), generator=torch.Generator().manual_seed(1)).to(cuda_device))
    q = torch.randn((B, d), generator=torch.Generator().manual_seed(2)).to(cuda_device)
    lists = [[5, 3, 9]] * B
    lists[17] = [1, 2, 3]
    sc = csr_from_lists(lists, cuda_device)
    assert isinstance(sc, SortedCSR)
    assert csr_sorted(sc) is sc
    s_ok, r_ok = ebt.score_topk(cat, k, queries=q, exclude=sc)
    raw_off = torch.tensor(np.arange(B + 1) * 3, dtype=torch.int64, device=cuda_device)
    raw_rows = torch.tensor(np.concatenate(lists), dtype=torch.int64, device=cuda_device)
    # through the Python layer a plain tuple is sorted first (ebt_sort_exclusions)
    s2, r2 = ebt.score_topk(cat, k, queries=q, exclude=(raw_off, raw_rows))
    assert torch.equal(r2, r_ok)
    # handed to the C entry unsorted: rejected by the rescore's check
    bad = SortedCSR(raw_off, raw_rows)     # a false claim: the rescore still checks
    with pytest.raises(L.EbertError, match="sorted ascending"):
        ebt.score_topk(cat, k, queries=q, exclude=bad)


@pytest.mark.parametrize("k", [20, 5999])
def test_non_finite_catalog_rows_never_candidates(cuda_device, k):
    """include/ebert.h "Non-finite catalog rows": a row with a NaN or an inf element scores NaN
    against every query and is never returned, on the screen path (k = 20) and the large-k
    full-sort path (k = 5999 > 4096, two slots left empty) alike; the rest keep the oracle order."""
    ebt, L = _ebt()
    n, d, B = 6000, 64, 4
    rng = np.random.default_rng(39)
    c = rng.standard_normal((n, d))
    q = rng.standard_normal((B, d))
    bad = [3, 1000, 4321]
    c[3, 5] = np.nan
    c[1000, 0] = np.inf
    c[4321] = q[0] * 10          # would be query 0's best row
    c[4321, 7] = np.nan
    cat = ebt.Catalog(torch.tensor(c, dtype=torch.float64, device=cuda_device))
    s, r = ebt.score_topk(cat, k, queries=torch.tensor(q, device=cuda_device))
    sn, rn = s.cpu().numpy(), r.cpu().numpy()
    good = np.setdiff1d(np.arange(n), bad)
    s_ref, r_ref = R.cosine_topk(q, c[good], min(k, len(good)))
    m = min(k, len(good))
    assert np.array_equal(rn[:, :m], good[r_ref])
    assert np.max(np.abs(sn[:, :m] - s_ref)) <= 1e-12
    assert not np.isin(rn, bad).any()
    assert np.all(rn[:, m:] == -1) and np.all(np.isnan(sn[:, m:]))


@pytest.mark.parametrize("k,batched", [(10, False), (10000, False), (10, True), (10000, True)])
def test_route_recommendations_matches_reference(cuda_device, k, batched):
    """Row a-1: GET /users/{user_id}/recommendations/?k= (api/users.py:150-155) through FastAPI's
    TestClient returns the reference's golden recommendations as JSON; the user without a liked
    movie gets HTTP 500 (the reference's uncaught sklearn ValueError), the one without ratings
    an empty list. batched: the route's scoring goes through a RecBatcher (§8f-2)."""
    from fastapi.testclient import TestClient
    from robot_ebert_amd import api
    from robot_ebert_amd.batcher import RecBatcher
    lib, gold = _collab_setup(cuda_device)
    b = RecBatcher(lib.movies_collab_catalog, max_batch=64, max_wait_ms=1.0) if batched else None
    client = TestClient(api.app(batcher=b), raise_server_exceptions=False)
    for uid, rec in gold["users"].items():
        want = rec[f"k{k}"]
        resp = client.get(f"/users/{uid}/recommendations/", params={"k": k})
        if isinstance(want, dict):
            assert resp.status_code == 500, (uid, resp.status_code)
            continue
        assert resp.status_code == 200, (uid, resp.text[:200])
        got = resp.json()
        assert [g["movie"]["tmdb_id"] for g in got] == [w[0] for w in want], uid
        np.testing.assert_allclose([g["score"] for g in got], [w[1] for w in want], rtol=0,
                                   atol=SCORE_ATOL)
        if not want:
            assert got == []
    if b is not None:
        b.close()
        api.app()   # the module-level route back to one call per request


@pytest.mark.parametrize("dt,d", [("f32", 1536), ("bf16", 768), ("f16", 200), ("f64", 64)])
def test_liked_prep_vector_form_bitwise(cuda_device, dt, d):
    """ebt_query_liked_sum's vector form (16-byte-aligned rows: staged row ids, eight liked rows'
    chunks in flight) writes exactly what the element form writes (same per-element order of
    additions): the same catalog once with aligned rows and once as a column slice of a wider
    matrix (ld = d + 1: the element form). Users with 0, 1 and 300 liked rows, duplicates."""
    ebt, L = _ebt()
    n = 20_000
    x = gaussian(51, n, d + 1, dt)
    wide = _t(x, dt, cuda_device)
    narrow = wide[:, :d].contiguous()
    cat_v = ebt.Catalog(narrow)                 # ld = d: the vector form
    cat_s = ebt.Catalog(wide[:, :d])            # ld = d + 1: the element form
    rng = np.random.default_rng(52)
    liked = [[5], rng.choice(n, 300, replace=False).tolist(), [7, 7, 19999],
             rng.choice(n, 17, replace=False).tolist()]
    from robot_ebert_amd.search import csr_from_lists
    lk = csr_from_lists(liked, cuda_device)
    assert cat_v.ld == d and cat_s.ld == d + 1
    # the same row norms for both (the norm kernel's own vector / element forms may round apart)
    cat_s.gnorm.copy_(cat_v.gnorm)
    qv = ebt.prepare_queries(cat_v, liked=lk)
    qs = ebt.prepare_queries(cat_s, liked=lk)
    assert torch.equal(qv.q64, qs.q64)
    assert torch.equal(qv.qimg.view(torch.int16), qs.qimg.view(torch.int16))
    assert torch.equal(qv.eps, qs.eps)


def test_rescore_row_count(cuda_device):
    """bench.py's roofline_topk counts the rows the rescore gathers inside the kernel
    (ebt_timer_count_rows): per query at least the k rows of pass A, at most the k' candidates,
    zero when counting is off, and the answer is the same with counting on."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd.search import plan
    dev = cuda_device
    c = torch.from_numpy(gaussian(31, 20000, 256, "f32").astype(np.float32)).to(dev)
    q = torch.from_numpy(gaussian(32, 512, 256, "f32").astype(np.float32)).to(dev)
    cat = ebt.Catalog(c)
    k = 50
    kp = plan(cat, 512, k)["kprime"]
    t = ebt.Timer()
    s0, r0 = ebt.score_topk(cat, k, queries=q, timer=t)
    torch.cuda.synchronize(dev)
    assert t.rows() == 0
    t.count_rows(True)
    t.reset()
    s1, r1 = ebt.score_topk(cat, k, queries=q, timer=t)
    torch.cuda.synchronize(dev)
    rows = t.rows()
    assert 512 * k <= rows <= 512 * kp, (rows, kp)
    assert torch.equal(r0, r1) and torch.equal(s0, s1)
    t.only("gemm")                      # the rescore stage not recorded: nothing counted
    t.reset()
    ebt.score_topk(cat, k, queries=q, timer=t)
    torch.cuda.synchronize(dev)
    assert t.rows() == 0
    t.count_rows(False)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_speculative_lead_equals_no_lead(cuda_device, dt):
    """The speculative screen's lead (C2's shape class: 100K rows x 4 query tiles -> 7 lead
    tiles whose hits come from the sample's stored scores, the filter over 6 whole rounds):
    the same rows AND scores as without the lead and as the unfused path, bit for bit, with
    exclusions; f32 (normalised f16 image) and native bf16 (row scales in the epilogue)."""
    ebt, L = _ebt()
    lib = L.load()
    n, d, B, k = 100_000, 128, 1024, 100
    c = gaussian(61, n, d, dt)
    q = gaussian(62, B, d, dt)
    rng = np.random.default_rng(63)
    excl = [list(np.sort(rng.choice(n, 30, replace=False))) for _ in range(B)]
    cat = ebt.Catalog(_t(c, dt, cuda_device))
    qt = _t(q, dt, cuda_device)
    sp = ebt.search.plan(cat, B, k)["spec"]
    assert sp is not None and sp["lead"] > 0, sp
    prev = lib.ebt_spec_lead(1)
    try:
        s1, r1 = ebt.score_topk(cat, k, queries=qt, exclude=excl)
        lib.ebt_spec_lead(0)
        assert ebt.search.plan(cat, B, k)["spec"]["lead"] == 0
        s0, r0 = ebt.score_topk(cat, k, queries=qt, exclude=excl)
    finally:
        lib.ebt_spec_lead(prev)
    s2, r2 = ebt.score_topk(cat, k, queries=qt, exclude=excl, fuse=False)
    assert torch.equal(r1, r0) and torch.equal(s1, s0)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(s1, s2, rtol=0, atol=0)
    idx = [0, 1, 511, 1023]
    s_ref, r_ref = R.cosine_topk(q[idx].astype(np.float64), c.astype(np.float64), k,
                                 [excl[i] for i in idx])
    assert_topk_equal(s1[idx], r1[idx], s_ref, r_ref)


def test_speculative_lead_hits_equal_filter_hits(cuda_device):
    """The lead tiles' hits (the pool GEMM's stored scores, taken by pool_kth_kernel) are the filter
    epilogue's own: a screen with the lead and one without give the same k best approx
    candidates (values and rows) for every query. (Past position k the lists may differ: later
    segments filter at the list's k-th - 2 eps, and the segments start at different rows.)"""
    ebt, L = _ebt()
    from robot_ebert_amd.search import prepare_queries, run_screen
    lib = L.load()
    n, d, B, k = 100_000, 64, 1024, 100
    c = gaussian(71, n, d, "f32")
    q = gaussian(72, B, d, "f32")
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    qb = prepare_queries(cat, queries=_t(q, "f32", cuda_device))
    kp = ebt.search.plan(cat, B, k)["kprime"]
    prev = lib.ebt_spec_lead(1)
    try:
        assert ebt.search.plan(cat, B, k)["spec"]["lead"] > 0
        lv1, lr1, ovf1, _ = run_screen(cat, qb, k, kp)
        lib.ebt_spec_lead(0)
        lv0, lr0, ovf0, _ = run_screen(cat, qb, k, kp)
    finally:
        lib.ebt_spec_lead(prev)
    # the wave merge writes a partitioned list: compare as sets of (value, row) per query
    a1 = torch.stack([lv1.view(torch.int32).to(torch.int64), lr1], -1).cpu().numpy()
    a0 = torch.stack([lv0.view(torch.int32).to(torch.int64), lr0], -1).cpu().numpy()
    for b in range(0, B, 7):   # positions [0, k): the k best of the partitioned list
        assert sorted(map(tuple, a1[b, :k])) == sorted(map(tuple, a0[b, :k])), b
    assert torch.equal(ovf1 != 0, ovf0 != 0)


def test_filter_split_launches_equal_one_launch(cuda_device):
    """A filter screen split into consecutive whole-round launches (ebt_filter_split: here 2
    tiles per workgroup, so a 100K-row x 1024-query segment runs as several launches) finds the
    same hits: the same final rows and scores as one launch per segment."""
    ebt, L = _ebt()
    lib = L.load()
    n, d, B, k = 100_000, 128, 1024, 50
    c = gaussian(81, n, d, "bf16")
    q = gaussian(82, B, d, "bf16")
    cat = ebt.Catalog(_t(c, "bf16", cuda_device))
    qt = _t(q, "bf16", cuda_device)
    prev = lib.ebt_filter_split(0)
    try:
        s0, r0 = ebt.score_topk(cat, k, queries=qt)
        lib.ebt_filter_split(2)
        t = ebt.Timer()
        s1, r1 = ebt.score_topk(cat, k, queries=qt, timer=t)
        assert t.query("gemm_filter")[1] >= 1
    finally:
        lib.ebt_filter_split(prev)
    assert torch.equal(r0, r1) and torch.equal(s0, s1)


def test_speculative_multi_segment_raise_in_merge(cuda_device):
    """A C3-shaped speculative screen (1M rows, 4096 queries, top-100; d = 64 to keep it cheap)
    runs several filter segments, each later one at the threshold the previous wave merge wrote
    (spec_threshold's RAISE folded into the merge, round 6), with exclusions looked up in every
    merge: the same rows and scores as the unfused path for all 4096 queries, bit for bit, and
    the float64 oracle on 32 of them."""
    ebt, L = _ebt()
    n, d, B, k = 1_000_000, 64, 4096, 100
    c = gaussian(71, n, d, "f32")
    q = gaussian(72, B, d, "f32")
    rng = np.random.default_rng(73)
    excl = [np.sort(rng.choice(n, 16, replace=False)) for _ in range(B)]
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    qt = _t(q, "f32", cuda_device)
    pl = ebt.search.plan(cat, B, k)
    assert pl["fused"] and pl["spec"] is not None, pl
    timer = ebt.Timer()
    ex = [list(e) for e in excl]
    s1, r1 = ebt.score_topk(cat, k, queries=qt, exclude=ex, timer=timer)
    merges = timer.query("merge_select")[1]
    assert merges >= 3, f"{merges} wave merges: the shape no longer runs several segments"
    s2, r2 = ebt.score_topk(cat, k, queries=qt, exclude=ex, fuse=False)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(s1, s2, rtol=0, atol=0)
    idx = np.linspace(0, B - 1, 32).round().astype(np.int64)
    s_ref, r_ref = R.cosine_topk(q[idx].astype(np.float64), c.astype(np.float64), k,
                                 [ex[i] for i in idx])
    ti = torch.from_numpy(idx).to(cuda_device)
    assert_topk_equal(s1[ti], r1[ti], s_ref, r_ref)
