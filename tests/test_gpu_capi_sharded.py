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


class Comm(ctypes.Structure):   # struct ebt_comm
    _fields_ = [("rank", I32), ("world", I32), ("n_global", I64), ("all_gather", GATHER),
                ("ctx", VP)]


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


def run_ranks(lib, hip, full, world, k, q=None, liked=None, excl=None, fail_rank=-1):
    """ebt_cosine_topk_sharded on `world` thread ranks; returns per-rank (rc, message, s, r)."""
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
        cb = GATHER(gather)
        comm = Comm(rank, world, n, cb, None)
        cat = cats[rank][0]
        B = q.shape[0] if q is not None else liked[0].numel() - 1
        need = lib.ebt_sharded_workspace_bytes(ctypes.byref(cat), ctypes.byref(comm), B, k, None)
        assert need > 0
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        s = torch.full((B, k), float("nan"), dtype=torch.float64, device=dev)
        rr = torch.full((B, k), -2, dtype=torch.int64, device=dev)
        lo, lr = liked if liked is not None else (None, None)
        eo, er = excl if excl is not None else (None, None)
        rc = lib.ebt_cosine_topk_sharded(
            ctypes.byref(cat), ctypes.byref(comm), P(q), CODE[q.dtype] if q is not None else 0, B,
            q.stride(0) if q is not None else 0, P(lo), P(lr), k, P(eo), P(er), None, P(ws), need,
            P(s), P(rr), None, torch.cuda.current_stream(dev).cuda_stream)
        msg = lib.ebt_last_error().decode() if rc else ""
        out[rank] = (rc, msg, s.cpu().numpy(), rr.cpu().numpy())
    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert all(o is not None for o in out), "a rank did not finish"
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
    assert calls == [4] * world          # threshold, floor, scores, rows
    s1, r1 = check_equal_single(lib, full, res, k, q=q, excl=ex)
    sample = [0, 150, 299]
    s_ref, r_ref = R.cosine_topk(qv[sample].astype(np.float32).astype(np.float64),
                                 c.astype(np.float32).astype(np.float64), k,
                                 [excl[i] for i in sample])
    np.testing.assert_array_equal(r1[sample], r_ref)
    np.testing.assert_allclose(s1[sample], s_ref, rtol=0, atol=1e-12)


def test_sharded_capi_large_k_block_merge(cuda_device, lib, hip):
    """3 uneven shards of a bf16 catalog, top-1000 (k' > 512: the floor-only branch with the block
    merge, no shared threshold); k > the smallest shard's rows is fine too."""
    n, d, B, k, world = 150_001, 256, 256, 1000, 3
    c = gaussian(211, n, d, "bf16")
    qv = gaussian(212, B, d, "bf16")
    full = torch.from_numpy(c).to(cuda_device).to(torch.bfloat16)
    q = torch.from_numpy(qv).to(cuda_device).to(torch.bfloat16)
    res, calls = run_ranks(lib, hip, full, world, k, q=q)
    assert calls == [3] * world          # floor, scores, rows
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
    assert calls == [4] * world          # partial sums, floor, scores, rows
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
