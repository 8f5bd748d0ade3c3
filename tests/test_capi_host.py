"""CPU: the C-ABI library loads and exports every declared symbol; host-side logic."""
import os
import re

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "ebert.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(ebt_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    import ctypes
    from robot_ebert_amd import _lib
    lib = _lib.load()
    syms = _declared_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib._SIGNATURES), set(syms) ^ set(_lib._SIGNATURES)
    assert lib.ebt_version() >= 200
    assert isinstance(lib.ebt_last_error(), bytes)


def test_invalid_args_return_einval_without_gpu():
    """Argument validation happens before any HIP call, so it is testable on the host."""
    from robot_ebert_amd import _lib
    lib = _lib.load()
    assert lib.ebt_select_topk(None, None, 0, 1, 0, 0, 0, 1, None, None, 0, None) == -1
    assert b"ebt_select_topk" in lib.ebt_last_error()
    assert lib.ebt_cosine_topk_workspace(10, 5, 100, 8, 128, 0) == 0  # B_pad < B
    assert lib.ebt_cosine_topk_workspace(10, 128, 1000, 104, 512, 0) > 0
    assert lib.ebt_merge_topk(None, None, 0, 1, 1, None, None, None) == -1


def test_compact_exchange_sizing_and_args_without_gpu():
    """The compact N > 1 exchange's sizing (ebt_shard_list_width, ebt_shard_pack_cap / _bytes)
    and argument checks are host code: C3/8 sends 27 entries per query for the floor and packs
    at most 27 results per query per rank; the compact form is off for one rank, for R k > 8192
    and for catalogs of 2^31 rows or more."""
    from robot_ebert_amd import _lib
    lib = _lib.load()
    assert lib.ebt_shard_list_width(100, 8) == 27          # ceil(1.5 * 100 / 8) + 8
    assert lib.ebt_shard_list_width(1000, 8) == 196
    assert lib.ebt_shard_list_width(7, 2) == 7             # never more than k
    cap = lib.ebt_shard_pack_cap(4096, 100, 8, 1_000_000)
    assert cap == 4096 * 27
    nb = lib.ebt_shard_pack_bytes(4096, cap)
    assert nb % 256 == 0 and nb >= 4 * (4096 + 1) + 12 * cap
    assert nb * 8 <= 12 * 2 ** 20                           # the results gather at C3/8 <= 12 MB
    assert lib.ebt_shard_pack_cap(4096, 100, 1, 1_000_000) == 0
    assert lib.ebt_shard_pack_cap(16, 2000, 8, 1_000_000) == 0
    assert lib.ebt_shard_pack_cap(16, 100, 8, 2 ** 31) == 0
    assert lib.ebt_shard_pack(None, None, 4, 10, None, 40, None, None) == -1
    assert b"ebt_shard_pack" in lib.ebt_last_error()
    assert lib.ebt_merge_packed(None, 8, 4, 10, 40, None, None, None, None) == -1
    assert lib.ebt_floor_pack(None, 10, 4, 10, 3, None, None, None) == -1
    assert lib.ebt_cosine_topk_sharded_finish(None) == -1
    assert lib.ebt_cosine_topk_sharded_wait(None) == -1


def test_workspace_grows_with_chunks():
    from robot_ebert_amd import _lib
    lib = _lib.load()
    one = lib.ebt_cosine_topk_workspace(4096, 4096, 1_000_000, 200, 1_000_064, 1)
    many = lib.ebt_cosine_topk_workspace(4096, 4096, 1_000_000, 200, 262_144, 1)
    fused = lib.ebt_cosine_topk_workspace(4096, 4096, 1_000_000, 200, 262_144, 0)
    assert one > 4096 * 1_000_000 * 4
    assert many < one
    assert fused < many  # the fused screen materialises only the head rows' scores


def test_self_contained_sizing_without_gpu():
    """ebt_catalog_state_bytes / ebt_workspace_bytes (the self-contained path's sizing) are host
    arithmetic: the catalog struct's device pointers are never dereferenced here."""
    import ctypes
    from robot_ebert_amd import _lib
    lib = _lib.load()
    n, d = 1_000_000, 1536
    f32 = lib.ebt_catalog_state_bytes(None, _lib.EBT_F32, n, d, d)
    assert f32 >= n * 8 + n * 4 + n * d * 2          # norms + inverse norms + f16 image
    aligned = 1 << 20                                # native f16, d % 64 == 0: no image copy
    assert lib.ebt_catalog_state_bytes(aligned, _lib.EBT_F16, n, d, d) < n * 16
    assert lib.ebt_catalog_state_bytes(None, _lib.EBT_F32, 0, d, d) == 0
    fake = 1 << 30
    cat = _lib.EbtCatalog(data=fake, dtype=_lib.EBT_F32, d=d, n=n, ld=d, row_offset=0,
                          gnorm64=fake, inv32=fake, image=fake, cscale=None,
                          img_dtype=_lib.EBT_F16, ld_img=d, d_pad=d, native=0, u_cat=2.0 ** -11)
    ws = lib.ebt_workspace_bytes(ctypes.byref(cat), 4096, 100, None)
    first = lib.ebt_cosine_topk_workspace(4096, 4096, n, 200, (4 << 30) // (4 * 4096) // 128 * 128, 0)
    assert ws > first > 0                            # first pass + retry area + prepared queries
    # k > 4096 < n: the full-sort path (large_k.hip, hand-written since round 6: its sizing is
    # host arithmetic too -- the CUB-compatible sort it replaced asked the device for its
    # temporaries, so without a GPU this used to read 0): two [Bg, n] (key, row) buffers
    big = lib.ebt_workspace_bytes(ctypes.byref(cat), 4096, 5000, None)
    assert big >= 2 * 12 * n
    bad = _lib.EbtOptions(kprime=0, flags=0, chunk_rows=100)                   # not % 128
    assert lib.ebt_workspace_bytes(ctypes.byref(cat), 4096, 100, ctypes.byref(bad)) == 0


def test_no_cpu_fallback_on_cpu_tensors():
    import torch
    from robot_ebert_amd import EbertError, Catalog
    with pytest.raises(EbertError):
        Catalog(torch.zeros((10, 4)))


def test_shard_range_partitions():
    from robot_ebert_amd.distributed import shard_range
    for n in (1, 7, 100, 2269, 1_000_000):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_split_liked_counts():
    from robot_ebert_amd.distributed import split_liked
    local, counts = split_liked([[1, 5, 9], [], [4]], 4, 9)
    assert local == [[5], [], [4]] and counts == [3, 0, 1]


def test_csr_from_lists_and_subset():
    import torch
    from robot_ebert_amd.search import csr_from_lists, csr_subset
    off, rows = csr_from_lists([[1, 2], [], [3, 4, 5]], "cpu")
    assert off.tolist() == [0, 2, 2, 5] and rows.tolist() == [1, 2, 3, 4, 5]
    o2, r2 = csr_subset(off, rows, torch.tensor([2, 0]))
    assert o2.tolist() == [0, 3, 5] and r2.tolist() == [3, 4, 5, 1, 2]
    o3, r3 = csr_subset(off, rows, torch.tensor([1]))
    assert o3.tolist() == [0, 0]


def test_order_recommendations_mirrors_reference():
    """lib.py:55 sort_index is lexicographic on string ids; lib.py:63 sort is stable."""
    from robot_ebert_amd.lib import order_recommendations
    pairs = [("9", 0.5), ("10", 0.7), ("100", 0.5), ("2", 0.9)]
    assert order_recommendations(pairs) == [("2", 0.9), ("10", 0.7), ("100", 0.5), ("9", 0.5)]


def test_user_query_lists():
    from robot_ebert_amd.lib import user_query_lists

    class FakeCat:
        row_offset = 0
        index_pos = {"a": 0, "b": 1, "c": 2}

        def rows_of(self, ids):
            return [self.index_pos[t] for t in ids]

    df = pd.DataFrame({"tmdb_id": ["a", "c", "b"], "rating": [3.5, 1.0, 5.0]})
    liked, rated = user_query_lists(df, FakeCat())
    assert liked == [0, 1] and sorted(rated) == [0, 1, 2]


def test_torch_ops_registered_with_fake_kernels():
    """torch.ops.ebert.* exist and trace on meta tensors (no GPU, no libebert call)."""
    import torch
    import robot_ebert_amd  # noqa: F401  (registers the ops)
    x = torch.empty(1000, 100, device="meta")
    g, inv = torch.ops.ebert.row_norms(x)
    assert g.shape == (1000,) and g.dtype == torch.float64 and inv.shape == (1024,)
    img = torch.ops.ebert.screen_image(x, g)
    assert img.shape == (1000, 128) and img.dtype == torch.float16
    q = torch.empty(7, 100, device="meta")
    s, r = torch.ops.ebert.cosine_topk(q, x, g, inv, img, 5, None, None, 0)
    assert s.shape == (7, 5) and r.dtype == torch.int64
    ms, mr = torch.ops.ebert.merge_topk(torch.empty(3, 7, 5, dtype=torch.float64, device="meta"),
                                        torch.empty(3, 7, 5, dtype=torch.int64, device="meta"), 5)
    assert ms.shape == (7, 5)


def test_spec_plan_poisson_rank():
    """The speculative screen's sample (ebt_cosine_topk_spec_plan): P evenly spaced tiles and the
    smallest rank j with P(Poisson(k' m / n) >= j) <= 1e-6 (api.hip:spec_params)."""
    import ctypes
    from scipy.stats import poisson
    from robot_ebert_amd import _lib
    lib = _lib.load()

    def sp(B, n, kp, flags=0):
        t, s, h = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        j = ctypes.c_int32()
        assert lib.ebt_cosine_topk_spec_plan(B, (B + 255) // 256 * 256 if B > 128 else 128, n,
                                             kp, flags, ctypes.byref(t), ctypes.byref(s),
                                             ctypes.byref(j), ctypes.byref(h)) == 0
        return t.value, s.value, j.value, h.value

    for (B, n, kp) in [(4096, 1_000_000, 200), (4096, 125_000, 200), (1024, 100_000, 120),
                       (4096, 250_000, 200)]:
        P, S, j, H = sp(B, n, kp)
        assert P >= 8 and P <= 64 and (P - 1) * S * 256 + 256 <= n
        lam = kp * 256 * P / n
        assert poisson.sf(j - 1, lam) <= 1e-6 < poisson.sf(j - 2, lam), (n, P, j)
        assert H >= j * n / (256 * P)
    assert sp(4096, 1_000_000, 200)[:3] == (16, 243, 9)    # round 5: 16 tiles (one pool round)
    assert sp(4096, 125_000, 200)[0] == 16          # one round of 256 workgroups
    assert sp(1024, 100_000, 120)[0] == 64          # C2: one workgroup per CU (64 tiles x 4)
    assert sp(100, 1_000_000, 104)[0] == 0          # B_pad = 128: the 128-tile kernel, no spec
    assert sp(4096, 1_000_000, 1016)[0] == 32       # k' <= 2048: spec with block merges
    assert sp(4096, 1_000_000, 2052)[0] == 0        # k' > 2048: no spec
    assert sp(4096, 20_000, 200)[0] == 0            # too few tiles for a sample
    assert sp(4096, 1_000_000, 200, _lib.EBT_FLAG_NO_FUSE)[0] == 0


def test_shared_threshold_plan():
    """The row-sharded path's shared threshold: spec_rank (Python) is the C rank rule, the
    sample size depends only on (n_global, world, B_pad) -- every rank takes the same decision
    before the all-gather -- and small batches / single ranks do not use it."""
    import ctypes
    from robot_ebert_amd import _lib
    from robot_ebert_amd.distributed import shard_range, shared_sample_tiles
    from robot_ebert_amd.search import spec_rank
    lib = _lib.load()
    for (n, kp) in [(1_000_000, 200), (125_000, 200), (6_250_000, 1256)]:
        t, s, h = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        j = ctypes.c_int32()
        assert lib.ebt_cosine_topk_spec_plan(4096, 4096, n, kp, 0, ctypes.byref(t),
                                             ctypes.byref(s), ctypes.byref(j),
                                             ctypes.byref(h)) == 0
        assert spec_rank(kp * 256 * t.value / n) == j.value
    assert shared_sample_tiles(1_000_000, 8, 4096) == 16     # one round of the sample GEMM
    assert shared_sample_tiles(1_000_000, 2, 4096) == 0       # 500K-row shards: own sample
    assert shared_sample_tiles(300_000, 2, 4096) == 16
    assert shared_sample_tiles(1_000_000, 1, 4096) == 0      # one rank: its own sample
    assert shared_sample_tiles(1_000_000, 8, 128) == 0       # B_pad 128: no pool epilogue
    assert shared_sample_tiles(20_000, 8, 4096) == 0         # shards too small to sample
    # every shard of shard_range holds the sample's tiles (stride >= 1)
    for world in (6, 7, 8):
        P = shared_sample_tiles(1_000_003, world, 4096)
        assert P > 0
        for r in range(world):
            a, b = shard_range(1_000_003, r, world)
            assert (b - a) // 256 >= P


def test_shared_sample_tiles_c_and_python_agree():
    """the sample's fill to one round of the persistent grid stays within the caps
    (<= 64 tiles per shard, world * 4 * tiles <= 2048 maxima per query, ebt_pool_kth's limit) in
    C (driver.hip sh_tiles, through ebt_shard_sample_tiles) and Python
    (distributed.shared_sample_tiles) alike: the two paths take the same decision for every
    config, e.g. B_pad = 512 on 8 ranks with 196K-300K-row shards (a round there is 128 tiles)."""
    from robot_ebert_amd import _lib
    from robot_ebert_amd.distributed import shared_sample_tiles
    lib = _lib.load()
    for world in (1, 2, 3, 4, 8, 16):
        for B_pad in (128, 256, 512, 1024, 2048, 4096, 16384):
            for n in (20_000, 100_000, 1_000_000, 1_570_000, 2_000_000, 2_400_000, 10_000_000):
                c = lib.ebt_shard_sample_tiles(n, world, B_pad)
                p = shared_sample_tiles(n, world, B_pad)
                assert c == p, (n, world, B_pad, c, p)
                assert 0 <= p <= 64 and world * 4 * p <= 2048
    assert shared_sample_tiles(8 * 250_000, 8, 512) > 0      # still shared, just not filled
    assert lib.ebt_shard_sample_tiles(0, 8, 512) == -1


def test_workspace_size_does_not_depend_on_the_lead_knob():
    """ebt_spec_lead changes whether the speculative sample's lead is used, never the workspace
    layout: a workspace sized with the knob in one state still fits the other (round 5)."""
    from robot_ebert_amd import _lib
    lib = _lib.load()
    prev = lib.ebt_spec_lead(1)
    try:
        for (B, n, kp) in [(1024, 100_000, 128), (4096, 1_000_000, 200), (4096, 125_000, 200)]:
            on = lib.ebt_cosine_topk_workspace(B, B, n, kp, 1 << 20, 0)
            lead_on = lib.ebt_cosine_topk_spec_lead(B, B, n, kp, 0)
            lib.ebt_spec_lead(0)
            off = lib.ebt_cosine_topk_workspace(B, B, n, kp, 1 << 20, 0)
            assert lib.ebt_cosine_topk_spec_lead(B, B, n, kp, 0) == 0
            lib.ebt_spec_lead(1)
            assert on == off > 0, (B, n, on, off)
            assert lead_on >= 0
        assert lib.ebt_cosine_topk_spec_lead(1024, 1024, 100_000, 128, 0) == 7   # C2
    finally:
        lib.ebt_spec_lead(prev)


def test_filter_split_default_and_set():
    """ebt_filter_split: long filter launches run as parts of at most 32 tiles per workgroup by
    default since 0.3.1 (512 before; profiles/r5/ab/tpw/), settable per process, 0 = never split;
    a negative argument only queries. Host code: no GPU call."""
    import os
    from robot_ebert_amd import _lib
    lib = _lib.load()
    cur = lib.ebt_filter_split(-1)
    if "EBT_FILTER_TPW" not in os.environ:
        assert cur == 32
    prev = lib.ebt_filter_split(64)
    try:
        assert prev == cur
        assert lib.ebt_filter_split(-1) == 64
        assert lib.ebt_filter_split(0) == 64
        assert lib.ebt_filter_split(-1) == 0
    finally:
        lib.ebt_filter_split(cur)
    assert lib.ebt_filter_split(-1) == cur


def test_sample_lead_argument_checks():
    """ebt_cosine_sample_lead (0.3.1) refuses, before any GPU call, a lead larger than the sample,
    sample tiles that run past the catalog, and a lead without its score buffer."""
    from robot_ebert_amd import _lib
    lib = _lib.load()
    n = 256 * 100

    def call(tiles, stride, lead, lead_scores, ld_lead):
        return lib.ebt_cosine_sample_lead(None, None, 256, None, None, 0, 64, n, 64, tiles,
                                          stride, None, 4 * tiles, lead, lead_scores, ld_lead,
                                          None, None)
    assert call(4, 2, 5, None, 0) == -1                        # lead > tiles
    assert b"ebt_cosine_sample" in lib.ebt_last_error()
    assert call(10, 12, 0, None, 0) == -1                      # last tile ends at row 256 * 109
    assert call(10, 11, 2, None, 512) == -1                    # lead without its scores
    assert call(0, 1, 0, None, 0) == -1 and call(4, 0, 0, None, 0) == -1
    assert call(4, 2, -1, None, 0) == -1


def _fake_catalog(n, d, dt):
    from robot_ebert_amd import _lib
    fake = 1 << 30
    native = dt in (_lib.EBT_F16, _lib.EBT_BF16)
    return _lib.EbtCatalog(data=fake, dtype=dt, d=d, n=n, ld=d, row_offset=0, gnorm64=fake,
                           inv32=fake, image=fake, cscale=fake if native else None,
                           img_dtype=dt if native else _lib.EBT_F16, ld_img=d, d_pad=d,
                           native=int(native), u_cat=0.0 if native else 2.0 ** -11)


@pytest.mark.parametrize("name,N,d,es,B,k", [("C4", 10_000_000, 768, 2, 8192, 100),
                                              ("C5", 50_000_000, 1536, 2, 16384, 1000),
                                              ("C3", 1_000_000, 1536, 4, 4096, 100)])
@pytest.mark.parametrize("all_reduce", [False, True])
def test_eight_gpu_memory_budget(name, N, d, es, B, k, all_reduce):
    """one rank of the 8-GPU step at the BASELINE shapes fits 0.8 x 288 GB by
    construction -- its shard, the catalog state (norms, inverse norms, image), ShardedTopk's
    default 3 slots of ebt_sharded_workspace_bytes, each slot's outputs and host buffer, and the
    query batch -- with or without the comm's float64 all-reduce (without it the liked path's
    partial sums are all-gathered: R x B x d x 8 more per slot). Host arithmetic only. Also pins
    the round-6 trim: the speculative screen's layout no longer carries the streaming select's
    chunk lists (C5/8 27.8 -> 13.0 GiB per slot)."""
    import ctypes
    from robot_ebert_amd import _lib
    lib = _lib.load()
    R = 8
    dt = {2: _lib.EBT_BF16 if name == "C4" else _lib.EBT_F16, 4: _lib.EBT_F32}[es]
    n = -(-N // R)
    shard = n * d * es
    state = lib.ebt_catalog_state_bytes(1 << 20, dt, n, d, d)
    assert state > 0
    cat = _fake_catalog(n, d, dt)
    cb = _lib.ALLGATHER_FN(lambda *a: 0)
    ar = _lib.ALLREDUCE_F64_FN(lambda *a: 0) if all_reduce else _lib.ALLREDUCE_F64_FN()
    comm = _lib.EbtComm(rank=0, world=R, n_global=N, all_gather=cb, all_reduce_f64=ar)
    ws = lib.ebt_sharded_workspace_bytes(ctypes.byref(cat), ctypes.byref(comm), B, k, None)
    assert ws > 0
    slots = 3
    outputs = slots * B * k * 16
    queries = B * d * es
    total = shard + state + slots * ws + outputs + queries
    assert total <= 0.8 * 288e9, (name, total / 1e9)
    if name == "C5":
        assert ws < 14 * 2 ** 30, ws / 2 ** 30          # was 27.76 GiB per slot (round 5)
        assert total < 70e9, total / 1e9
