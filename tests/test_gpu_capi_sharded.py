"""GPU: the row-sharded self-contained C entry (include/ebert.h ebt_cosine_topk_sharded) through a
bare ctypes binding, the way a non-Python host would bind it -- ranks simulated by threads on one
MI355X, each with its own shard (an ebt_catalog whose row_offset is the shard's first global row)
and an all-gather callback that exchanges device buffers through hipMemcpy (the role RCCL's
ncclAllGather plays on an 8-GPU node). The protocol -- shared screening
threshold, catalog-wide floor, local retries, gather + merge -- runs inside libebert; every
rank's answer must equal ONE ebt_cosine_topk over the whole catalog (rows bit-exact, scores
equal) and the float64 oracle on sampled queries. Reference: /root/reference/src/backend/app/
lib.py:51-55 (per shard) and :32-63 (the liked-rows mean, the rated-rows exclusion).
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

from inputs import gaussian
from oracle import restatement as R
from test_gpu_capi import CODE, LIB, P, Catalog, csr, make_catalog, topk

pytestmark = pytest.mark.gpu
VP, I32, I64, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
GATHER = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP, VP, SZ, VP)


class Comm(ctypes.Structure):   # struct ebt_comm (all_reduce_f64 left NULL: the gather path)
    _fields_ = [("rank", I32), ("world", I32), ("n_global", I64), ("all_gather", GATHER),
                ("ctx", VP), ("all_reduce_f64", VP)]


class Options(ctypes.Structure):   # struct ebt_options
    _fields_ = [("kprime", I32), ("flags", I32), ("chunk_rows", I64)]


class Pending(ctypes.Structure):   # struct ebt_pending
    _fields_ = [("cat", VP), ("opt", Options), ("B", I64), ("B_pad", I64), ("chunk", I64),
                ("k", I32), ("k_eff", I32), ("kprime", I32), ("flags", I32), ("excl_off", VP),
                ("excl_rows", VP), ("ws", VP), ("ws_bytes", SZ), ("out_scores", VP),
                ("out_rows", VP), ("cert_host", VP), ("event", VP), ("timer", VP),
                ("stream", VP)]


class ShardedPending(ctypes.Structure):   # struct ebt_sharded_pending
    _fields_ = [("local", Pending), ("comm", Comm), ("out_scores", VP), ("out_rows", VP),
                ("host", VP), ("event", VP), ("stage", I32)]


@pytest.fixture(scope="module")
def lib():
    h = ctypes.CDLL(LIB)
    h.ebt_last_error.restype = ctypes.c_char_p
    h.ebt_catalog_state_bytes.argtypes = [VP, ctypes.c_int, I64, I32, I64]
    h.ebt_catalog_state_bytes.restype = SZ
    h.ebt_catalog_init.argtypes = [ctypes.POINTER(Catalog), VP, ctypes.c_int, I64, I32, I64, I64,
                                   VP, SZ, VP]
    h.ebt_workspace_bytes.argtypes = [ctypes.POINTER(Catalog), I64, I32, VP]
    h.ebt_workspace_bytes.restype = SZ
    h.ebt_cosine_topk.argtypes = [ctypes.POINTER(Catalog), VP, ctypes.c_int, I64, I64, VP, VP,
                                  I32, VP, VP, VP, VP, SZ, VP, VP, VP, VP]
    h.ebt_sharded_workspace_bytes.argtypes = [ctypes.POINTER(Catalog), ctypes.POINTER(Comm), I64,
                                              I32, VP]
    h.ebt_sharded_workspace_bytes.restype = SZ
    h.ebt_cosine_topk_sharded.argtypes = [ctypes.POINTER(Catalog), ctypes.POINTER(Comm), VP,
                                          ctypes.c_int, I64, I64, VP, VP, I32, VP, VP, VP, VP, SZ,
                                          VP, VP, VP, VP]
    h.ebt_cosine_topk_sharded_submit.argtypes = [
        ctypes.POINTER(Catalog), ctypes.POINTER(Comm), VP, ctypes.c_int, I64, I64, VP, VP, I32,
        VP, VP, VP, VP, SZ, VP, VP, VP, ctypes.POINTER(ShardedPending), VP, VP]
    h.ebt_cosine_topk_sharded_finish.argtypes = [ctypes.POINTER(ShardedPending)]
    h.ebt_cosine_topk_sharded_wait.argtypes = [ctypes.POINTER(ShardedPending)]
    return h


@pytest.fixture(scope="module")
def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipMemcpy.argtypes = [VP, VP, SZ, ctypes.c_int]
    h.hipStreamSynchronize.argtypes = [VP]
    return h


def shard_cuts(n, world):
    base, rem = divmod(n, world)
    cuts = [0]
    for r in range(world):
        cuts.append(cuts[-1] + base + (1 if r < rem else 0))
    return cuts


REDUCE = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP, SZ, VP)


def run_ranks(lib, hip, full, world, k, q=None, liked=None, excl=None, fail_rank=-1,
              allreduce=False, opt=None):
    """ebt_cosine_topk_sharded on `world` thread ranks; returns per-rank (rc, message, s, r).
    allreduce: the comm also offers all_reduce_f64 (a barrier exchange summing in rank order)."""
    dev = full.device
    n = full.shape[0]
    cuts = shard_cuts(n, world)
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world, timeout=120),
              "calls": [0] * world, "rslots": [None] * world, "reduces": [0] * world}
    cats = []
    for r in range(world):
        cat, state = make_catalog(lib, full[cuts[r]:cuts[r + 1]])
        cat.row_offset = cuts[r]
        cats.append((cat, state))
    out = [None] * world

    def body(rank):
        def gather(ctx, send, recv, nbytes, stream):
            try:
                shared["calls"][rank] += 1
                if rank == fail_rank:
                    shared["barrier"].abort()
                    return -7
                hip.hipStreamSynchronize(stream)           # send is complete
                shared["slots"][rank] = send
                shared["barrier"].wait()
                for src in range(world):
                    if hip.hipMemcpy(recv + src * nbytes, shared["slots"][src], nbytes, 3):
                        return -1
                shared["barrier"].wait()                   # nobody reuses send before all copied
                return 0
            except threading.BrokenBarrierError:
                return -9
        def reduce(ctx, buf, count, stream):
            try:
                shared["reduces"][rank] += 1
                hip.hipStreamSynchronize(stream)
                mine = torch.empty(count, dtype=torch.float64, device=dev)
                if hip.hipMemcpy(mine.data_ptr(), buf, count * 8, 3):
                    return -1
                shared["rslots"][rank] = mine
                shared["barrier"].wait()
                acc = shared["rslots"][0].clone()
                for src in range(1, world):
                    acc += shared["rslots"][src]
                torch.cuda.synchronize(dev)
                if hip.hipMemcpy(buf, acc.data_ptr(), count * 8, 3):
                    return -1
                shared["barrier"].wait()
                return 0
            except threading.BrokenBarrierError:
                return -9
        cb = GATHER(gather)
        rcb = REDUCE(reduce)
        comm = Comm(rank, world, n, cb, None, ctypes.cast(rcb, VP) if allreduce else None)
        cat = cats[rank][0]
        B = q.shape[0] if q is not None else liked[0].numel() - 1
        optp = ctypes.byref(opt) if opt is not None else None
        need = lib.ebt_sharded_workspace_bytes(ctypes.byref(cat), ctypes.byref(comm), B, k, optp)
        assert need > 0
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        s = torch.full((B, k), float("nan"), dtype=torch.float64, device=dev)
        rr = torch.full((B, k), -2, dtype=torch.int64, device=dev)
        lo, lr = liked if liked is not None else (None, None)
        eo, er = excl if excl is not None else (None, None)
        rc = lib.ebt_cosine_topk_sharded(
            ctypes.byref(cat), ctypes.byref(comm), P(q), CODE[q.dtype] if q is not None else 0, B,
            q.stride(0) if q is not None else 0, P(lo), P(lr), k, P(eo), P(er), optp, P(ws), need,
            P(s), P(rr), None, torch.cuda.current_stream(dev).cuda_stream)
        msg = lib.ebt_last_error().decode() if rc else ""
        out[rank] = (rc, msg, s.cpu().numpy(), rr.cpu().numpy())
    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert all(o is not None for o in out), "a rank did not finish"
    if allreduce:
        return out, shared["calls"], shared["reduces"]
    return out, shared["calls"]


def check_equal_single(lib, full, res, k, q=None, liked=None, excl=None):
    cat, state = make_catalog(lib, full)
    rc, s1, r1 = topk(lib, cat, k, full.device, q=q, liked=liked, excl=excl)
    assert rc == 0, lib.ebt_last_error()
    for rank, (rc, msg, s, r) in enumerate(res):
        assert rc == 0, (rank, msg)
        np.testing.assert_array_equal(r, r1)
        m = r1 >= 0
        np.testing.assert_array_equal(s[m], s1[m])
        assert np.all(np.isnan(s[~m]))
    return s1, r1


def test_sharded_capi_shared_threshold_exclusions(cuda_device, lib, hip):
    """4 ranks of 100K rows (the shared-threshold branch), f32 catalog, 300 queries, top-50,
    150 excluded rows per query drawn partly from each query's true top 100."""
    n, d, B, k, world = 400_000, 128, 300, 50, 4
    c = gaussian(201, n, d, "f32")
    qv = gaussian(202, B, d, "f32")
    s0, r0 = R.cosine_topk(qv[:4], c, 100)
    rng = np.random.default_rng(203)
    excl = [np.unique(np.concatenate([r0[b % 4, rng.choice(100, 20, replace=False)],
                                      rng.choice(n, 130, replace=False)])) for b in range(B)]
    full = torch.from_numpy(c.astype(np.float32)).to(cuda_device)
    q = torch.from_numpy(qv.astype(np.float32)).to(cuda_device)
    ex = csr(excl, cuda_device)
    res, calls = run_ranks(lib, hip, full, world, k, q=q, excl=ex)
    assert calls == [3] * world          # threshold, floor, packed results
    s1, r1 = check_equal_single(lib, full, res, k, q=q, excl=ex)
    sample = [0, 150, 299]
    s_ref, r_ref = R.cosine_topk(qv[sample].astype(np.float32).astype(np.float64),
                                 c.astype(np.float32).astype(np.float64), k,
                                 [excl[i] for i in sample])
    np.testing.assert_array_equal(r1[sample], r_ref)
    np.testing.assert_allclose(s1[sample], s_ref, rtol=0, atol=1e-12)


def test_sharded_capi_local_retries_repack(cuda_device, lib, hip):
    """Round 6: the sharded rescore counts each query's packed entries and one launch places
    them -- unless the shard's local retries rewrote some list, when the finish packs again with
    the two-launch ebt_shard_pack. Forced here: k' = k on 2 ranks of 350K rows (no shared
    threshold: every shard's list holds k' candidates, so no query is certified at k' = k and
    every query is retried at k' x 4); the answer equals the single-GPU path's at default
    options and the float64 oracle."""
    n, d, B, k, world = 700_000, 64, 256, 20, 2
    c = gaussian(221, n, d, "f32")
    qv = gaussian(222, B, d, "f32")
    full = torch.from_numpy(c.astype(np.float32)).to(cuda_device)
    q = torch.from_numpy(qv.astype(np.float32)).to(cuda_device)
    res, calls = run_ranks(lib, hip, full, world, k, q=q, opt=Options(k, 0, 0))
    assert calls == [2] * world          # floor, packed results (no threshold at 350K rows)
    s1, r1 = check_equal_single(lib, full, res, k, q=q)
    s_ref, r_ref = R.cosine_topk(qv[[0, 255]].astype(np.float32).astype(np.float64),
                                 c.astype(np.float32).astype(np.float64), k)
    np.testing.assert_array_equal(r1[[0, 255]], r_ref)


def test_sharded_capi_large_k_block_merge(cuda_device, lib, hip):
    """3 uneven shards of a bf16 catalog, top-1000 (k' > 512: the floor-only branch with the block
    merge, no shared threshold); k > the smallest shard's rows is fine too."""
    n, d, B, k, world = 150_001, 256, 256, 1000, 3
    c = gaussian(211, n, d, "bf16")
    qv = gaussian(212, B, d, "bf16")
    full = torch.from_numpy(c).to(cuda_device).to(torch.bfloat16)
    q = torch.from_numpy(qv).to(cuda_device).to(torch.bfloat16)
    res, calls = run_ranks(lib, hip, full, world, k, q=q)
    assert calls == [2] * world          # floor, packed results
    s1, r1 = check_equal_single(lib, full, res, k, q=q)
    c64 = full[:].double().cpu().numpy()
    q64 = q.double().cpu().numpy()
    s_ref, r_ref = R.cosine_topk(q64[[0, 255]], c64, k)
    np.testing.assert_array_equal(r1[[0, 255]], r_ref)


def test_sharded_capi_liked_users(cuda_device, lib, hip):
    """The collaborative path: liked rows spread over the shards (each sums its own, one
    all-gather of the float64 partial sums), rated rows excluded, k larger than a shard; the
    sklearn ValueError text for a user without a liked movie, on every rank alike."""
    n, d, k, world = 30_000, 64, 40, 3
    c = gaussian(221, n, d, "f64")
    liked = [[1, 2, 29_999], [10_000], [5, 6_000, 12_000, 29_995], [20_001, 20_002]]
    rated = [sorted(set(x) | {7, 8, 29_980}) for x in liked]
    full = torch.from_numpy(c).to(cuda_device)
    lk, ex = csr(liked, cuda_device), csr(rated, cuda_device)
    res, calls = run_ranks(lib, hip, full, world, k, liked=lk, excl=ex)
    assert calls == [3] * world          # partial sums, floor, packed results
    s1, r1 = check_equal_single(lib, full, res, k, liked=lk, excl=ex)
    want_s, want_r = R.liked_topk(c, liked, k, rated)
    np.testing.assert_array_equal(r1, want_r)
    np.testing.assert_allclose(s1, want_s, rtol=0, atol=1e-12)
    bad = csr([[1, 2], []], cuda_device)
    res, calls = run_ranks(lib, hip, full, world, k, liked=bad)
    for rc, msg, _, _ in res:
        assert rc != 0 and "Found array with 0 sample(s)" in msg
    assert calls == [0] * world          # detected before the first collective


def test_sharded_capi_collective_failure(cuda_device, lib, hip):
    """A failing all-gather on one rank fails the call on every rank with EBT_EHIP and the
    callback's status in the message (the others see their barrier broken), never a hang."""
    n, d, B, k, world = 60_000, 64, 64, 10, 2
    c = gaussian(231, n, d, "f32")
    full = torch.from_numpy(c.astype(np.float32)).to(cuda_device)
    q = torch.from_numpy(gaussian(232, B, d, "f32").astype(np.float32)).to(cuda_device)
    res, _ = run_ranks(lib, hip, full, world, k, q=q, fail_rank=1)
    for rc, msg, _, _ in res:
        assert rc == -2 and "all_gather returned" in msg


def run_ranks_pipelined(lib, hip, full, world, k, batches, n_ws=3):
    """ebt_cosine_topk_sharded_submit / _finish / _wait on `world` thread ranks with batches in
    flight: per step submit(i), finish(i-1), wait(i-2) (the order include/ebert.h suggests),
    `n_ws` workspaces cycled. Returns per rank the list of (scores, rows) per batch and the
    all-gather calls per rank."""
    dev = full.device
    n = full.shape[0]
    cuts = shard_cuts(n, world)
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world, timeout=120),
              "calls": [0] * world}
    cats = []
    for r in range(world):
        cat, state = make_catalog(lib, full[cuts[r]:cuts[r + 1]])
        cat.row_offset = cuts[r]
        cats.append((cat, state))
    out = [None] * world
    errs = []

    def body(rank):
        try:
            def gather(ctx, send, recv, nbytes, stream):
                try:
                    shared["calls"][rank] += 1
                    hip.hipStreamSynchronize(stream)
                    shared["slots"][rank] = send
                    shared["barrier"].wait()
                    for src in range(world):
                        if hip.hipMemcpy(recv + src * nbytes, shared["slots"][src], nbytes, 3):
                            return -1
                    shared["barrier"].wait()
                    return 0
                except threading.BrokenBarrierError:
                    return -9
            cb = GATHER(gather)
            comm = Comm(rank, world, n, cb, None)
            cat = cats[rank][0]
            B = batches[0].shape[0]
            need = lib.ebt_sharded_workspace_bytes(ctypes.byref(cat), ctypes.byref(comm), B, k,
                                                   None)
            assert need > 0
            wss = [torch.empty(need, dtype=torch.uint8, device=dev) for _ in range(n_ws)]
            hosts = [torch.zeros(B + 2, dtype=torch.int32).pin_memory() for _ in range(n_ws)]
            pend = [ShardedPending() for _ in range(n_ws)]
            res = [(torch.empty((B, k), dtype=torch.float64, device=dev),
                    torch.empty((B, k), dtype=torch.int64, device=dev)) for _ in batches]
            st = torch.cuda.current_stream(dev).cuda_stream

            def check(rc, what):
                if rc:
                    raise AssertionError(f"rank {rank} {what}: {lib.ebt_last_error().decode()}")
            nb = len(batches)
            for i in range(nb + 2):
                if i < nb:
                    q, w = batches[i], i % n_ws
                    check(lib.ebt_cosine_topk_sharded_submit(
                        ctypes.byref(cat), ctypes.byref(comm), P(q), CODE[q.dtype], B, q.stride(0),
                        None, None, k, None, None, None, P(wss[w]), need, P(res[i][0]),
                        P(res[i][1]), P(hosts[w]), ctypes.byref(pend[w]), None, st), "submit")
                if 1 <= i <= nb:
                    check(lib.ebt_cosine_topk_sharded_finish(ctypes.byref(pend[(i - 1) % n_ws])),
                          "finish")
                if 2 <= i:
                    check(lib.ebt_cosine_topk_sharded_wait(ctypes.byref(pend[(i - 2) % n_ws])),
                          "wait")
            torch.cuda.synchronize(dev)
            out[rank] = [(s.cpu().numpy(), r.cpu().numpy()) for s, r in res]
        except Exception as e:  # noqa: BLE001 -- reported after the join
            errs.append(e)
            shared["barrier"].abort()
    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert not errs, errs
    assert all(o is not None for o in out), "a rank did not finish"
    return out, shared["calls"]


def test_sharded_capi_pipelined_eight_ranks(cuda_device, lib, hip):
    """Eight thread ranks, four batches in flight through submit / finish / wait (three
    workspaces): every rank's answer for every batch equals ONE ebt_cosine_topk over the whole
    catalog, and the step issues three all-gathers (threshold, floor, packed results)."""
    n, d, B, k, world = 800_000, 128, 512, 100, 8
    c = gaussian(241, n, d, "f32")
    full = torch.from_numpy(c.astype(np.float32)).to(cuda_device)
    batches = [torch.from_numpy(gaussian(242 + i, B, d, "f32").astype(np.float32)).to(cuda_device)
               for i in range(4)]
    res, calls = run_ranks_pipelined(lib, hip, full, world, k, batches)
    assert calls == [3 * len(batches)] * world
    cat, state = make_catalog(lib, full)
    for i, q in enumerate(batches):
        rc, s1, r1 = topk(lib, cat, k, cuda_device, q=q)
        assert rc == 0, lib.ebt_last_error()
        for rank in range(world):
            s, r = res[rank][i]
            np.testing.assert_array_equal(r, r1)
            np.testing.assert_array_equal(s, s1)
    s_ref, r_ref = R.cosine_topk(gaussian(242, B, d, "f32")[[0, 511]].astype(np.float32)
                                 .astype(np.float64), c.astype(np.float32).astype(np.float64), k)
    rc, s1, r1 = topk(lib, cat, k, cuda_device, q=batches[0])
    np.testing.assert_array_equal(r1[[0, 511]], r_ref)


def test_sharded_capi_packed_overflow_falls_back(cuda_device, lib, hip):
    """Skewed data: every query's whole top 50 lives on shard 0 (noisy copies of the queries),
    so shard 0's entries above the floor exceed its packed capacity (ceil(1.5 k / R) + 8 per
    query on average): the merge flags the batch incomplete and _wait re-merges from the full
    lists (two more all-gathers on every rank) -- the answer stays exact."""
    n, d, B, k, world = 80_000, 64, 128, 50, 4
    rng = np.random.default_rng(251)
    qv = rng.standard_normal((B, d))
    c = rng.standard_normal((n, d))
    near = np.repeat(qv, 156, axis=0) + 0.3 * rng.standard_normal((156 * B, d))
    c[:156 * B] = near                    # inside shard 0 = rows [0, 20000)
    full = torch.from_numpy(c.astype(np.float32)).to(cuda_device)
    q = torch.from_numpy(qv.astype(np.float32)).to(cuda_device)
    res, calls = run_ranks(lib, hip, full, world, k, q=q)
    assert calls == [4] * world           # floor, packed, then scores + rows
    s1, r1 = check_equal_single(lib, full, res, k, q=q)
    assert np.all(r1[:, :k] < 20_000)
    s_ref, r_ref = R.cosine_topk(qv[[0, 77]].astype(np.float32).astype(np.float64),
                                 c.astype(np.float32).astype(np.float64), k)
    np.testing.assert_array_equal(r1[[0, 77]], r_ref)


def test_sharded_capi_unsorted_liked(cuda_device, lib, hip):
    """Liked rows out of order, or several on a later shard (include/ebert.h: the shards'
    partial sums group the additions by shard): the reference's rows, scores within float64
    round-off of the oracle (which averages the per-row cosines, lib.py:51-52)."""
    n, d, k, world = 30_000, 64, 40, 3
    c = gaussian(261, n, d, "f64")
    liked = [[29_999, 1, 2], [20_002, 10_000, 5], [12_000, 6_000, 29_995, 3],
             [1, 10_001, 10_002, 10_003, 20_004, 20_005]]
    full = torch.from_numpy(c).to(cuda_device)
    off = torch.tensor([0, 3, 6, 10, 16], dtype=torch.int64, device=cuda_device)
    rows = torch.tensor(sum(liked, []), dtype=torch.int64, device=cuda_device)
    res, calls = run_ranks(lib, hip, full, world, k, liked=(off, rows))
    want_s, want_r = R.liked_topk(c, liked, k, [[] for _ in liked])
    for rc, msg, s, r in res:
        assert rc == 0, msg
        np.testing.assert_array_equal(r, want_r)
        np.testing.assert_allclose(s, want_s, rtol=0, atol=1e-12)


def test_sharded_capi_liked_all_reduce(cuda_device, lib, hip):
    """The liked path over a comm that offers all_reduce_f64 (RCCL's ncclAllReduce on a node):
    the partial sums go through one all-reduce instead of an all-gather (here a barrier
    exchange summing in rank order, the gather path's order, so the answer is the gather path's
    bit for bit) and the workspace drops the gathered-sums buffer."""
    n, d, k, world = 30_000, 64, 40, 3
    c = gaussian(221, n, d, "f64")
    liked = [[1, 2, 29_999], [10_000], [5, 6_000, 12_000, 29_995], [20_001, 20_002]]
    rated = [sorted(set(x) | {7, 8, 29_980}) for x in liked]
    full = torch.from_numpy(c).to(cuda_device)
    lk, ex = csr(liked, cuda_device), csr(rated, cuda_device)
    res, calls, reduces = run_ranks(lib, hip, full, world, k, liked=lk, excl=ex, allreduce=True)
    assert calls == [2] * world and reduces == [1] * world   # floor, packed; the partial sums
    s1, r1 = check_equal_single(lib, full, res, k, liked=lk, excl=ex)
    want_s, want_r = R.liked_topk(c, liked, k, rated)
    np.testing.assert_array_equal(r1, want_r)
    cat, state = make_catalog(lib, full[:10_000])
    g = Comm(0, world, n, GATHER(lambda *a: 0), None, None)
    g2 = Comm(0, world, n, GATHER(lambda *a: 0), None, ctypes.cast(REDUCE(lambda *a: 0), VP))
    need_g = lib.ebt_sharded_workspace_bytes(ctypes.byref(cat), ctypes.byref(g), 4096, k, None)
    need_r = lib.ebt_sharded_workspace_bytes(ctypes.byref(cat), ctypes.byref(g2), 4096, k, None)
    assert need_g - need_r >= world * 4096 * d * 8
