"""GPU: the self-contained C ABI (include/ebert.h: ebt_catalog_init, ebt_workspace_bytes,
ebt_cosine_topk) driven through a bare ctypes binding, the way a non-Python caller (cgo / JNI /
N-API) would bind it -- no robot_ebert_amd import; torch only allocates device memory.

Every golden case the reference produced (tests/golden: sklearn cosine_similarity + pandas sort
top-k for nine seeded shapes / dtypes, and get_user_recs of /root/reference/src/backend/app/
lib.py:32-63 for the 20 C1 users) must come out of ONE ebt_cosine_topk call per batch: rows
bit-exact, scores within 1e-12, the sklearn ValueError text for a user without liked movies.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from inputs import COS_CASES, c1_catalog, cos_case_inputs
from oracle import restatement as R

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "robot_ebert_amd", "libebert.so")
TDT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}
VP, I32, I64, SZ, F32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t,
                         ctypes.c_float)


class Catalog(ctypes.Structure):   # struct ebt_catalog
    _fields_ = [("data", VP), ("dtype", I32), ("d", I32), ("n", I64), ("ld", I64),
                ("row_offset", I64), ("gnorm64", VP), ("inv32", VP), ("image", VP),
                ("cscale", VP), ("img_dtype", I32), ("ld_img", I32), ("d_pad", I32),
                ("native", I32), ("u_cat", F32)]


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
    return h


def P(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def make_catalog(lib, emb: torch.Tensor):
    st = torch.cuda.current_stream(emb.device).cuda_stream
    n, d = emb.shape
    need = lib.ebt_catalog_state_bytes(P(emb), CODE[emb.dtype], n, d, emb.stride(0))
    state = torch.empty(need, dtype=torch.uint8, device=emb.device)
    cat = Catalog()
    rc = lib.ebt_catalog_init(ctypes.byref(cat), P(emb), CODE[emb.dtype], n, d, emb.stride(0), 0,
                              P(state), need, st)
    assert rc == 0, lib.ebt_last_error()
    return cat, state


def csr(lists, dev):
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(x) for x in lists])
    flat = np.concatenate([np.sort(np.asarray(x, dtype=np.int64)) for x in lists]) \
        if off[-1] else np.zeros(1, dtype=np.int64)
    return torch.from_numpy(off).to(dev), torch.from_numpy(flat).to(dev)


def topk(lib, cat, k, dev, q=None, liked=None, excl=None):
    """One ebt_cosine_topk call; returns (rc, scores, rows)."""
    B = q.shape[0] if q is not None else liked[0].numel() - 1
    ws_bytes = lib.ebt_workspace_bytes(ctypes.byref(cat), B, k, None)
    assert ws_bytes > 0
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    s = torch.empty((B, k), dtype=torch.float64, device=dev)
    r = torch.empty((B, k), dtype=torch.int64, device=dev)
    lo, lr = liked if liked is not None else (None, None)
    eo, er = excl if excl is not None else (None, None)
    rc = lib.ebt_cosine_topk(ctypes.byref(cat), P(q), CODE[q.dtype] if q is not None else 0, B,
                             q.stride(0) if q is not None else 0, P(lo), P(lr), k, P(eo), P(er),
                             None, P(ws), ws_bytes, P(s), P(r), None,
                             torch.cuda.current_stream(dev).cuda_stream)
    return rc, s.cpu().numpy(), r.cpu().numpy()


@pytest.mark.parametrize("name", sorted(COS_CASES))
def test_capi_cos_topk_golden(cuda_device, lib, name):
    case = COS_CASES[name]
    q, c, excl = cos_case_inputs(case)
    gold = np.load(os.path.join(GOLD, "cos_topk_small.npz"))
    dt = TDT[case["dtype"]]
    emb = torch.from_numpy(c).to(cuda_device).to(dt)
    qt = torch.from_numpy(q).to(cuda_device).to(dt)
    cat, state = make_catalog(lib, emb)
    rc, s, r = topk(lib, cat, case["k"], cuda_device, q=qt,
                    excl=csr(excl, cuda_device) if excl is not None else None)
    assert rc == 0, lib.ebt_last_error()
    r_ref = gold[f"{name}_rows"].astype(np.int64)
    np.testing.assert_array_equal(r, r_ref)
    m = r_ref >= 0
    np.testing.assert_allclose(s[m], gold[f"{name}_scores"][m], rtol=0, atol=1e-12)


@pytest.mark.parametrize("k", [10, 10000])
def test_capi_user_recs_golden(cuda_device, lib, k):
    """get_user_recs (lib.py:32-63) for the 20 C1 users: liked rows -> mean cosine query,
    rated rows excluded; one batched call for every user with a liked movie, the sklearn
    ValueError text (via ebt_last_error) for the user without one, [] for no ratings."""
    with open(os.path.join(GOLD, "c1_collab.json")) as f:
        gold = json.load(f)
    ids, c = c1_catalog()
    pos = {t: i for i, t in enumerate(ids)}
    emb = torch.from_numpy(c).to(cuda_device)          # float64, as constants.py:56
    cat, state = make_catalog(lib, emb)
    users, liked, rated, want = [], [], [], []
    for uid, rec in gold["users"].items():
        ratings = [(t, r) for t, r in rec["ratings"] if t in pos]       # lib.py:44
        w = rec[f"k{k}"]
        if not rec["ratings"]:
            assert w == []                                              # lib.py:39-40
            continue
        li = [pos[t] for t, r in ratings if r >= 3.5]                   # lib.py:47
        ra = [pos[t] for t, r in ratings]                               # lib.py:48
        if isinstance(w, dict):                                         # no liked movie
            rc, _, _ = topk(lib, cat, k, cuda_device, liked=csr([li], cuda_device),
                            excl=csr([ra], cuda_device))
            assert rc == -1
            assert lib.ebt_last_error().decode() == w["message"]
            continue
        users.append(uid)
        liked.append(li)
        rated.append(ra)
        want.append(w)
    rc, s, r = topk(lib, cat, k, cuda_device, liked=csr(liked, cuda_device),
                    excl=csr(rated, cuda_device))
    assert rc == 0, lib.ebt_last_error()
    for b, (uid, w) in enumerate(zip(users, want)):
        m = r[b] >= 0
        got_ids = [ids[i] for i in r[b][m]]
        assert got_ids == [x[0] for x in w], uid
        np.testing.assert_allclose(s[b][m], [x[1] for x in w], rtol=0, atol=1e-12)
        assert np.all(np.isnan(s[b][~m]))


def test_capi_errors(cuda_device, lib):
    """Unsorted exclusions and out-of-catalog liked rows fail loudly (EBT_EINVAL)."""
    emb = torch.randn((1000, 64), device=cuda_device)
    cat, state = make_catalog(lib, emb)
    q = torch.randn((4, 64), device=cuda_device)
    off = torch.tensor([0, 2, 2, 2, 2], dtype=torch.int64, device=cuda_device)
    rows = torch.tensor([9, 3], dtype=torch.int64, device=cuda_device)   # unsorted segment
    rc, _, _ = topk(lib, cat, 10, cuda_device, q=q, excl=(off, rows))
    assert rc == -1 and b"sorted" in lib.ebt_last_error()
    rc, _, _ = topk(lib, cat, 10, cuda_device, liked=csr([[1, 5000]], cuda_device))
    assert rc == -1 and b"not in the catalog" in lib.ebt_last_error()


def test_capi_memory_errors(cuda_device, lib):
    """Every buffer is the caller's: an undersized state or workspace fails with EBT_ENOMEM
    (-3) and the needed size in the message, before any kernel runs; invalid sizes make
    ebt_workspace_bytes return 0; the catalog stays usable afterwards."""
    dev = cuda_device
    emb = torch.randn((6000, 64), device=dev)
    n, d = emb.shape
    st = torch.cuda.current_stream(dev).cuda_stream
    need = lib.ebt_catalog_state_bytes(P(emb), CODE[emb.dtype], n, d, d)
    small = torch.empty(need - 256, dtype=torch.uint8, device=dev)
    c0 = Catalog()
    rc = lib.ebt_catalog_init(ctypes.byref(c0), P(emb), CODE[emb.dtype], n, d, d, 0, P(small),
                              need - 256, st)
    assert rc == -3 and b"state" in lib.ebt_last_error()
    cat, state = make_catalog(lib, emb)
    # any k: min(k, n) > 4096 takes the full-sort path (tests/test_gpu_large_k.py)
    assert lib.ebt_workspace_bytes(ctypes.byref(cat), 4, 5000, None) > 0
    assert lib.ebt_workspace_bytes(ctypes.byref(cat), 4, 7000, None) > 0
    assert lib.ebt_workspace_bytes(ctypes.byref(cat), 4, 4096, None) > 0
    assert lib.ebt_workspace_bytes(ctypes.byref(cat), 0, 10, None) == 0    # invalid batch
    q = torch.randn((4, d), device=dev)
    k = 10
    ws_bytes = lib.ebt_workspace_bytes(ctypes.byref(cat), 4, k, None)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    s = torch.full((4, k), -7.0, dtype=torch.float64, device=dev)
    r = torch.full((4, k), -7, dtype=torch.int64, device=dev)
    rc = lib.ebt_cosine_topk(ctypes.byref(cat), P(q), CODE[q.dtype], 4, d, None, None, k, None,
                             None, None, P(ws), ws_bytes - 1, P(s), P(r), None, st)
    assert rc == -3 and b"workspace" in lib.ebt_last_error()
    torch.cuda.synchronize(dev)
    assert (s == -7.0).all() and (r == -7).all()          # nothing was written
    rc, s2, r2 = topk(lib, cat, k, dev, q=q)
    assert rc == 0 and (r2 >= 0).all()


def test_workspace_allocation_failure_is_loud(cuda_device):
    """The Python surface allocates the workspace with torch: when it cannot, the caller gets
    torch's OutOfMemoryError (no partial result, no fallback), and the next call succeeds."""
    import robot_ebert_amd as ebt
    dev = cuda_device
    cat = ebt.Catalog(torch.randn((200_000, 256), device=dev))
    q = torch.randn((4096, 256), device=dev)
    free, total = torch.cuda.mem_get_info(dev)
    used = torch.cuda.memory_allocated(dev)
    torch.cuda.empty_cache()
    # leave room for what is allocated now plus 1 MiB: the batch's workspace cannot fit
    torch.cuda.set_per_process_memory_fraction((used + (1 << 20)) / total, dev)
    try:
        with pytest.raises(torch.OutOfMemoryError):
            ebt.score_topk(cat, 100, queries=q)
    finally:
        torch.cuda.set_per_process_memory_fraction(1.0, dev)
    s, r = ebt.score_topk(cat, 100, queries=q[:8])
    assert (r >= 0).all()


@pytest.mark.parametrize("buffer", ["pinned", "pageable"])
def test_capi_submit_certificates_pinned_or_pageable(cuda_device, lib, buffer):
    """ebt_cosine_topk_submit / _finish with the certificate buffer in pinned host memory (the
    rescore writes it itself, ABI 0.3.3) or in pageable memory (a copy from the workspace):
    both deliver every certificate and the same exact answer. A clustered catalog makes some
    first-pass certificates 0 / -1, so the retries read what was delivered; a buffer left at a
    non-certificate value would have failed the finish with EBT_EHIP."""
    dev = cuda_device
    rng = np.random.default_rng(29)
    n, d, B, k, C = 60_000, 64, 256, 50, 16
    centers = rng.standard_normal((C, d))
    x = (centers[rng.integers(0, C, n)] + 0.03 * rng.standard_normal((n, d))).astype(np.float32)
    qv = (centers[rng.integers(0, C, B)] + 0.015 * rng.standard_normal((B, d))).astype(np.float32)
    emb = torch.from_numpy(x).to(dev)
    q = torch.from_numpy(qv).to(dev)
    cat, state = make_catalog(lib, emb)
    lib.ebt_cosine_topk_submit.argtypes = [ctypes.POINTER(Catalog), VP, ctypes.c_int, I64, I64,
                                           VP, VP, I32, VP, VP, VP, VP, SZ, VP, VP, VP, VP, VP,
                                           VP]
    lib.ebt_cosine_topk_finish.argtypes = [VP]
    ws_bytes = lib.ebt_workspace_bytes(ctypes.byref(cat), B, k, None)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    s = torch.empty((B, k), dtype=torch.float64, device=dev)
    r = torch.empty((B, k), dtype=torch.int64, device=dev)
    if buffer == "pinned":
        cert_t = torch.full((B + 1,), 9, dtype=torch.int32, pin_memory=True)
        cert_np, cert_p = cert_t.numpy(), ctypes.c_void_p(cert_t.data_ptr())
    else:
        cert_np = np.full(B + 1, 9, dtype=np.int32)
        cert_p = cert_np.ctypes.data_as(VP)
    pend = ctypes.create_string_buffer(1024)            # struct ebt_pending (opaque here)
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = lib.ebt_cosine_topk_submit(ctypes.byref(cat), P(q), CODE[q.dtype], B, d, None, None, k,
                                    None, None, None, P(ws), ws_bytes, P(s), P(r), cert_p, pend,
                                    None, st)
    assert rc == 0, lib.ebt_last_error()
    rc = lib.ebt_cosine_topk_finish(pend)
    assert rc == 0, lib.ebt_last_error()
    first = cert_np[:B].copy()                          # the first pass's, as delivered
    assert set(np.unique(first)) <= {1, 0, -1}, np.unique(first)
    assert (first != 1).any(), "no retry exercised"
    s_ref, r_ref = R.cosine_topk(qv.astype(np.float64), x.astype(np.float64), k)
    np.testing.assert_array_equal(r.cpu().numpy(), r_ref)
    np.testing.assert_allclose(s.cpu().numpy(), s_ref, rtol=0, atol=1e-12)
