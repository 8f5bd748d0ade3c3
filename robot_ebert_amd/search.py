"""Query x catalog cosine top-k on the GPU: the replacement of ``lib.py:51-55``.

    pairwise_similarities = cosine_similarity(catalog.loc[liked], catalog)      # lib.py:51
    movie_scores = pd.Series(pairwise_similarities.mean(axis=0), ...)           # lib.py:52
    recommended = movie_scores.loc[unrated].sort_values(ascending=False)[:k]    # lib.py:55

``score_topk`` takes a batch of queries -- either dense vectors (the L = 1 case, BASELINE
configs C2-C5) or per-user lists of liked catalog rows (the collaborative path, folded into one
query vector per user: q = mean_l normalize(x_l), lib.py:51-52) -- plus optional per-query
excluded rows (the rated movies, lib.py:48,55), and returns the top-k (score desc, row asc) with
float64 scores equal to the reference's float64 arithmetic.

Pipeline (all on the caller's current HIP stream, see include/ebert.h):
  query prep -> [per catalog chunk: MFMA screening GEMM -> mask excluded -> streaming top-k'
  select] -> select across chunks -> exact float64 rescore + certification. Queries whose
candidate set cannot be certified (a tie cluster wider than k' at the k-th score) are re-run
with a 4x larger k'; there is no CPU fallback.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib
from ._lib import DTYPE_CODE, EbertError, call, ptr, region, require_cuda, stream_of
from .catalog import Catalog

KPRIME_MAX = 4096
QUERY_PREP_MAX_D = 4096  # ebt_query_prep keeps 16 elements per thread
MERGE_WAVE_KMAX = 512   # largest k' of the fused wave-merge screen (select_topk.hip WMERGE_K)
DEFAULT_SCORE_BUDGET = int(os.environ.get("EBT_SCORE_BUDGET", str(4 << 30)))  # bytes of f32 scores


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def pad_batch(B: int) -> int:
    """Query rows of the MFMA image: the 256x256-tile GEMM serves batches above 128 queries,
    the 128x128-tile one smaller batches (ebt_screen_scores picks by B_pad % 256)."""
    B = max(B, 1)
    return _round_up(B, 128) if B <= 128 else _round_up(B, 256)


@dataclass
class QueryBatch:
    """Device-side prepared queries (ebt_query_* outputs)."""
    q64: torch.Tensor      # [B, d] float64 (normalised query / mean of normalised liked rows)
    qimg: torch.Tensor     # [B_pad, ld_img] f16/bf16 MFMA operand
    qscale: torch.Tensor   # [B_pad] float32 epilogue scale
    eps: torch.Tensor      # [B_pad] float32 certification bound
    B: int

    @property
    def B_pad(self) -> int:
        return int(self.qimg.shape[0])

    def subset(self, idx: torch.Tensor) -> "QueryBatch":
        n = int(idx.numel())
        B_pad = pad_batch(n)
        qimg = torch.zeros((B_pad, self.qimg.shape[1]), dtype=self.qimg.dtype, device=self.qimg.device)
        qimg[:n] = self.qimg.index_select(0, idx)
        qscale = torch.ones(B_pad, dtype=torch.float32, device=self.qimg.device)
        qscale[:n] = self.qscale.index_select(0, idx)
        eps = torch.zeros(B_pad, dtype=torch.float32, device=self.qimg.device)
        eps[:n] = self.eps.index_select(0, idx)
        return QueryBatch(self.q64.index_select(0, idx).contiguous(), qimg, qscale, eps, n)


class SortedCSR(tuple):
    """(offsets, rows) of a device CSR the library built with every segment sorted ascending
    (csr_from_lists, csr_sorted): passed back as `exclude`, it is used as it is -- no re-sort per
    call. (The rescore checks each segment's order anyway, folded into the kernel that writes the
    certificates: an unsorted segment fails the call, it is never silently misread.)"""

    # host facts of a CSR built from host lists (None when unknown): the shortest segment and
    # the row range, so that a liked CSR can be passed with EBT_FLAG_LIKED_CHECKED
    min_len = None
    row_min = None
    row_max = None

    def __new__(cls, off: torch.Tensor, rows: torch.Tensor, min_len=None, row_min=None,
                row_max=None):
        t = super().__new__(cls, (off, rows))
        t.min_len, t.row_min, t.row_max = min_len, row_min, row_max
        return t

    def checked_for(self, lo: int, hi: int) -> bool:
        """Every segment non-empty and every row in [lo, hi) (known from the host build)."""
        return (self.min_len is not None and self.min_len >= 1 and self.row_min is not None
                and self.row_min >= lo and self.row_max < hi)


def csr_from_lists(lists: Sequence[Sequence[int]], device,
                   stager=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Host lists of row ids -> device CSR (offsets int64 [B+1], rows int64 [nnz]), each segment
    sorted (ebt_cosine_topk_prepared binary-searches them). numpy builds it (a batch of a few
    thousand users' lists costs the interpreter ~1 ms as Python loops, on the serving path's
    dispatcher thread) and ONE host-to-device copy moves offsets and rows together."""
    segs = [np.sort(np.asarray(l, dtype=np.int64).ravel()) for l in lists]
    lens = np.fromiter((x.size for x in segs), dtype=np.int64, count=len(segs))
    B = len(segs)
    both = np.empty(B + 1 + max(int(lens.sum()), 1), dtype=np.int64)
    both[0] = 0
    np.cumsum(lens, out=both[1:B + 1])
    if lens.sum():
        np.concatenate(segs, out=both[B + 1:])
    else:
        both[B + 1] = 0
    # (with a hostio.HostStager the copy runs on its copy stream from pinned memory, under the
    # kernels of the batch before; the compute stream waits for it)
    t = stager.to_device(both) if stager is not None else torch.from_numpy(both).to(device)
    nnz = int(lens.sum())
    rows = both[B + 1:B + 1 + nnz]
    return SortedCSR(t[:B + 1], t[B + 1:], min_len=int(lens.min()) if B else 0,
                     row_min=int(rows.min()) if nnz else None,
                     row_max=int(rows.max()) if nnz else None)


def csr_sorted(off, rows: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """A caller's device CSR with every segment sorted ascending (the fused merge drops excluded
    rows by binary search over the segment, so an unsorted segment would silently keep rated
    rows): ebt_sort_exclusions, the library's own segmented sort. Offsets are absolute positions
    into `rows` (off[0] may be > 0); positions outside every segment keep their value. Returns
    (off, sorted copy of rows) as a SortedCSR (a caller may keep it and pass it on every call)."""
    if isinstance(off, SortedCSR):   # csr_sorted(*sorted_csr) or csr_sorted(sorted_csr)
        return off
    require_cuda(off, "exclusion offsets")
    require_cuda(rows, "exclusion rows")
    if off.dtype != torch.int64 or rows.dtype != torch.int64:
        raise EbertError("exclusion CSR must be int64 (offsets, rows)")
    off, rows = off.contiguous(), rows.contiguous()
    nnz = int(rows.numel())
    B = int(off.numel()) - 1
    if nnz <= 1 or B < 1:
        return SortedCSR(off, rows)
    need = _lib.load().ebt_sort_exclusions_bytes(B, nnz)
    if need == 0:
        raise EbertError(f"exclusion CSR of {B} segments / {nnz} rows cannot be sorted")
    ws = torch.empty(need, dtype=torch.uint8, device=rows.device)
    out = torch.empty_like(rows)
    call("ebt_sort_exclusions", ptr(off), ptr(rows), ptr(out), B, nnz, ptr(ws), need,
         stream_of(rows.device))
    return SortedCSR(off, out)


def csr_subset(off: torch.Tensor, rows: torch.Tensor, idx: torch.Tensor):
    """Rows `idx` of a device CSR (torch ops only; used for the certification retry)."""
    starts = off.index_select(0, idx)
    lens = off.index_select(0, idx + 1) - starts
    new_off = torch.zeros(idx.numel() + 1, dtype=torch.int64, device=off.device)
    new_off[1:] = torch.cumsum(lens, 0)
    total = int(new_off[-1].item())
    if total == 0:
        return new_off, torch.zeros(1, dtype=torch.int64, device=off.device)
    seg = torch.repeat_interleave(torch.arange(idx.numel(), device=off.device), lens)
    pos = torch.arange(total, device=off.device) - new_off[:-1].index_select(0, seg)
    return new_off, rows.index_select(0, starts.index_select(0, seg) + pos)


def prepare_queries(catalog: Catalog, queries: Optional[torch.Tensor] = None,
                    liked: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                    liked_counts: Optional[torch.Tensor] = None,
                    liked_sum_hook=None) -> QueryBatch:
    """Build q64 / qimg / qscale / eps for a batch.

    queries : dense [B, d] CUDA tensor (any supported dtype), or
    liked   : device CSR (offsets [B+1], LOCAL rows) of liked catalog rows per user; the query is
              sum_l x_l/||x_l|| divided by liked_counts (default: the CSR lengths). liked_sum_hook,
              if given, is applied to the float64 sums before the division (the cross-shard
              all-reduce of a row-sharded catalog).
    """
    dev = catalog.device
    st = stream_of(dev)
    d = catalog.d
    if (queries is None) == (liked is None):
        raise EbertError("pass exactly one of queries= or liked=")
    native_q = False
    if queries is not None:
        require_cuda(queries, "queries")
        if queries.dim() != 2 or queries.shape[1] != d:
            raise EbertError(f"queries must be [B, {d}], got {tuple(queries.shape)}")
        if queries.dtype not in DTYPE_CODE:
            raise EbertError(f"unsupported query dtype {queries.dtype}")
        if queries.stride(1) != 1:
            queries = queries.contiguous()
        B = int(queries.shape[0])
        q64 = torch.empty((B, d), dtype=torch.float64, device=dev)
        native_q = catalog.native and queries.dtype == catalog.img_torch_dtype
        if d <= QUERY_PREP_MAX_D:   # one launch: q64, image, scale and eps (ebt_query_prep)
            B_pad = pad_batch(B)
            qimg = torch.empty((B_pad, catalog.ld_img), dtype=catalog.img_torch_dtype, device=dev)
            qscale = torch.empty(B_pad, dtype=torch.float32, device=dev)
            eps = torch.empty(B_pad, dtype=torch.float32, device=dev)
            call("ebt_query_prep", ptr(queries), DTYPE_CODE[queries.dtype], B, B_pad, d,
                 int(queries.stride(0)), catalog.img_dtype, 1 if native_q else 0,
                 float(catalog.u_cat), ptr(q64), ptr(qimg), catalog.ld_img, ptr(qscale),
                 ptr(eps), st)
            return QueryBatch(q64, qimg, qscale, eps, B)
        call("ebt_query_dense", ptr(queries), DTYPE_CODE[queries.dtype], B, d,
             int(queries.stride(0)), ptr(q64), st)
    else:
        off, rows = liked
        B = int(off.numel()) - 1
        q64 = torch.empty((B, d), dtype=torch.float64, device=dev)
        local = rows - catalog.row_offset if catalog.row_offset else rows
        call("ebt_query_liked_sum", ptr(catalog.data), catalog.dtype_code, d, catalog.ld,
             ptr(catalog.gnorm), B, ptr(off), ptr(local), ptr(q64), st)
        if liked_sum_hook is not None:
            q64 = liked_sum_hook(q64)
        counts = liked_counts if liked_counts is not None else (off[1:] - off[:-1])
        if bool((counts <= 0).any().item()):
            raise ValueError(
                f"Found array with 0 sample(s) (shape=(0, {d})) while a minimum of 1 is required "
                "by check_pairwise_arrays.")
        scale = (1.0 / counts.to(torch.float64)).contiguous()
        call("ebt_scale_rows_f64", ptr(q64), B, d, ptr(scale), st)
    B_pad = pad_batch(B)
    qimg = torch.empty((B_pad, catalog.ld_img), dtype=catalog.img_torch_dtype, device=dev)
    qscale = torch.empty(B_pad, dtype=torch.float32, device=dev)
    eps = torch.empty(B_pad, dtype=torch.float32, device=dev)
    call("ebt_query_image", ptr(q64), B, B_pad, d, catalog.img_dtype,
         ptr(queries) if native_q else None, int(queries.stride(0)) if native_q else 0,
         1 if native_q else 0, float(catalog.u_cat), ptr(qimg), catalog.ld_img, ptr(qscale),
         ptr(eps), st)
    return QueryBatch(q64, qimg, qscale, eps, B)


def default_kprime(catalog: Catalog, k: int) -> int:
    """Screening width: native images have a tiny error bound, f16 images need more slack.
    The rows inside the 2 eps band around the k-th score grow with k (Gaussian tail: about
    2 eps k z sqrt(d) of them, z ~ 4): at C5 (k = 1000, d = 1536, native f16) ~55, so the
    native slack is k / 4, at least 16."""
    kp = k + max(16, k // 4) if catalog.native else max(2 * k, k + 32)
    return min(_round_up(kp, 8), KPRIME_MAX)


def _chunk_rows(catalog: Catalog, B_pad: int, budget: int) -> int:
    rows = budget // (4 * B_pad)
    rows = max(128, rows // 128 * 128)
    return min(rows, _round_up(catalog.n, 128))


def plan(catalog: Catalog, B: int, k: int, kprime: Optional[int] = None,
         chunk_rows: Optional[int] = None, fuse: bool = True) -> dict:
    """How score_topk will run a batch of B queries (ebt_cosine_topk_plan): k', fused or not,
    head rows (screened through the materialised-score path), largest fused tail segment (rows),
    chunk rows."""
    import ctypes
    B_pad = pad_batch(B)
    k_eff = min(k, catalog.n)
    kp = kprime or default_kprime(catalog, k_eff)
    kp = max(_round_up(k_eff, 4), min(_round_up(kp, 4), _round_up(catalog.n, 4), KPRIME_MAX))
    chunk = chunk_rows or _chunk_rows(catalog, B_pad, DEFAULT_SCORE_BUDGET)
    h, c, ch = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    f = ctypes.c_int32()
    call("ebt_cosine_topk_plan", B, B_pad, catalog.n, kp, chunk,
         0 if fuse else _lib.EBT_FLAG_NO_FUSE, ctypes.byref(h), ctypes.byref(c), ctypes.byref(ch),
         ctypes.byref(f))
    out = {"kprime": kp, "B_pad": B_pad, "fused": bool(f.value), "head_rows": h.value,
           "segment_rows_max": c.value, "chunk_rows": ch.value}
    out["spec"] = spec_plan(B, catalog.n, kp, fuse)
    return out


def spec_plan(B: int, n: int, kprime: int, fuse: bool = True) -> Optional[dict]:
    """The speculative screen's sample (ebt_cosine_topk_spec_plan) or None when not used:
    tiles (256 rows each), stride (tiles apart, from tile 0), rank (j) and expected hits."""
    import ctypes
    t, st, h = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
    j = ctypes.c_int32()
    call("ebt_cosine_topk_spec_plan", B, pad_batch(B), n, kprime,
         0 if fuse else _lib.EBT_FLAG_NO_FUSE, ctypes.byref(t), ctypes.byref(st), ctypes.byref(j),
         ctypes.byref(h))
    if t.value == 0:
        return None
    lead = int(_lib.load().ebt_cosine_topk_spec_lead(B, pad_batch(B), n, kprime,
                                                     0 if fuse else _lib.EBT_FLAG_NO_FUSE))
    return {"tiles": t.value, "stride": st.value, "rank": j.value, "hits": round(h.value, 1),
            "lead": lead}


def run_pipeline(catalog: Catalog, qb: QueryBatch, k: int, kprime: int,
                 exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                 chunk_rows: Optional[int] = None, timer: Optional[_lib.Timer] = None,
                 workspace: Optional[torch.Tensor] = None, flags: int = 0):
    """One ebt_cosine_topk_prepared call. Returns (scores f64 [B,k], rows i64 [B,k], certified i32 [B]);
    certified is 1 (exact), 0 (widen k') or -1 (fused candidate list overflowed: run unfused)."""
    dev = catalog.device
    st = stream_of(dev)
    B, B_pad = qb.B, qb.B_pad
    chunk = chunk_rows or _chunk_rows(catalog, B_pad, DEFAULT_SCORE_BUDGET)
    need = _lib.load().ebt_cosine_topk_workspace(B, B_pad, catalog.n, kprime, chunk, flags)
    if need == 0:
        raise EbertError("invalid workspace request")
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    cert = torch.empty(B, dtype=torch.int32, device=dev)
    eo, er = (exclude if exclude is not None else (None, None))
    call("ebt_cosine_topk_prepared", ptr(qb.q64), ptr(qb.qimg), ptr(qb.qscale), ptr(qb.eps), B, B_pad,
         ptr(catalog.data), catalog.dtype_code, catalog.ld, ptr(catalog.gnorm), ptr(catalog.image),
         ptr(catalog.cscale), catalog.img_dtype, catalog.ld_img, catalog.n, catalog.d,
         catalog.d_pad, catalog.row_offset, ptr(eo), ptr(er), k, kprime, chunk, flags, ptr(workspace),
         int(workspace.numel()), ptr(out_s), ptr(out_r), ptr(cert),
         timer.handle if timer is not None else None, st)
    return out_s, out_r, cert


def run_screen(catalog: Catalog, qb: QueryBatch, k: int, kprime: int,
               exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
               chunk_rows: Optional[int] = None, timer: Optional[_lib.Timer] = None,
               flags: int = 0):
    """Phase 1 of the two-phase sharded top-k (ebt_cosine_screen): this shard's k' best approx
    candidates. Returns (vals f32 [B,k'], GLOBAL rows i64 [B,k'], ovf i32 [B], eps f32 [B])."""
    dev = catalog.device
    B, B_pad = qb.B, qb.B_pad
    chunk = chunk_rows or _chunk_rows(catalog, B_pad, DEFAULT_SCORE_BUDGET)
    need = _lib.load().ebt_cosine_topk_workspace(B, B_pad, catalog.n, kprime, chunk, flags)
    if need == 0:
        raise EbertError("invalid workspace request")
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    lv = torch.empty((B, kprime), dtype=torch.float32, device=dev)
    lr = torch.empty((B, kprime), dtype=torch.int64, device=dev)
    ovf = torch.empty(B, dtype=torch.int32, device=dev)
    eps = torch.empty(B, dtype=torch.float32, device=dev)
    eo, er = (exclude if exclude is not None else (None, None))
    call("ebt_cosine_screen", ptr(qb.q64), ptr(qb.qimg), ptr(qb.qscale), ptr(qb.eps), B, B_pad,
         ptr(catalog.data), catalog.dtype_code, catalog.ld, ptr(catalog.gnorm), ptr(catalog.image),
         ptr(catalog.cscale), catalog.img_dtype, catalog.ld_img, catalog.n, catalog.d,
         catalog.d_pad, catalog.row_offset, ptr(eo), ptr(er), k, kprime, chunk, flags, ptr(ws),
         int(ws.numel()), ptr(lv), ptr(lr), ptr(ovf), ptr(eps),
         timer.handle if timer is not None else None, stream_of(dev))
    return lv, lr, ovf, eps


def spec_rank(lam: float, tail: float = 1e-6) -> int:
    """The smallest j with P(Poisson(lam) >= j) <= tail (api.hip spec_params): the rank of the
    sample maxima whose value exceeds the k'-th best catalog score with probability <= tail."""
    import math
    pmf, cdf, j = math.exp(-lam), 0.0, 0
    while j < 100000 and 1.0 - cdf > tail:
        cdf += pmf
        pmf *= lam / (j + 1)
        j += 1
    return max(j, 1)


def sample_maxima(catalog: Catalog, qb: QueryBatch, tiles: int,
                  timer: Optional[_lib.Timer] = None) -> torch.Tensor:
    """ebt_cosine_sample: `tiles` evenly spaced full 256-row tiles of this catalog (shard)
    through the screening GEMM, keeping the max of every 64-row subgroup: [B_pad, 4 tiles] f32."""
    stride = (catalog.n // 256) // tiles
    if stride > 1 and stride % 2 == 0:  # odd, as ebt_cosine_topk_prepared's own sample (api.hip)
        stride -= 1
    out = torch.empty((qb.B_pad, 4 * tiles), dtype=torch.float32, device=catalog.device)
    call("ebt_cosine_sample", ptr(qb.qimg), ptr(qb.qscale), qb.B_pad, ptr(catalog.image),
         ptr(catalog.cscale), catalog.img_dtype, catalog.ld_img, catalog.n, catalog.d_pad, tiles,
         stride, ptr(out), 4 * tiles, timer.handle if timer is not None else None,
         stream_of(catalog.device))
    return out


def pool_kth(pooled: torch.Tensor, B: int, B_pad: int, j: int) -> torch.Tensor:
    """ebt_pool_kth: theta[b] = the j-th largest of pooled[b, :] ([B, G] f32, G <= 2048);
    +inf for the padding rows B <= b < B_pad."""
    pooled = pooled.contiguous()
    theta = torch.empty(B_pad, dtype=torch.float32, device=pooled.device)
    call("ebt_pool_kth", ptr(pooled), pooled.shape[1], B, B_pad, pooled.shape[1], j, ptr(theta),
         stream_of(pooled.device))
    return theta


def screen_at(catalog: Catalog, qb: QueryBatch, k: int, kprime: int, theta: torch.Tensor,
              hits: float, exclude: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
              chunk_rows: Optional[int] = None, timer: Optional[_lib.Timer] = None):
    """ebt_cosine_screen_at: run_screen at the caller's threshold theta [B_pad] f32 (see
    include/ebert.h: the caller verifies theta against the catalog-wide floor)."""
    dev = catalog.device
    B, B_pad = qb.B, qb.B_pad
    chunk = chunk_rows or _chunk_rows(catalog, B_pad, DEFAULT_SCORE_BUDGET)
    need = _lib.load().ebt_cosine_topk_workspace(B, B_pad, catalog.n, kprime, chunk,
                                                 _lib.EBT_FLAG_THETA)
    if need == 0:
        raise EbertError("invalid workspace request")
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    lv = torch.empty((B, kprime), dtype=torch.float32, device=dev)
    lr = torch.empty((B, kprime), dtype=torch.int64, device=dev)
    ovf = torch.empty(B, dtype=torch.int32, device=dev)
    eps = torch.empty(B, dtype=torch.float32, device=dev)
    eo, er = (exclude if exclude is not None else (None, None))
    call("ebt_cosine_screen_at", ptr(qb.q64), ptr(qb.qimg), ptr(qb.qscale), ptr(qb.eps), B,
         B_pad, ptr(catalog.data), catalog.dtype_code, catalog.ld, ptr(catalog.gnorm),
         ptr(catalog.image), ptr(catalog.cscale), catalog.img_dtype, catalog.ld_img, catalog.n,
         catalog.d, catalog.d_pad, catalog.row_offset, ptr(eo), ptr(er), k, kprime, chunk, 0,
         ptr(ws), int(ws.numel()), ptr(lv), ptr(lr), ptr(ovf), ptr(eps), ptr(theta.contiguous()),
         float(hits), timer.handle if timer is not None else None, stream_of(dev))
    return lv, lr, ovf, eps


def score_topk_submit(catalog: Catalog, k: int, queries: Optional[torch.Tensor] = None,
               liked: Optional[Union[Tuple[torch.Tensor, torch.Tensor], Sequence[Sequence[int]]]] = None,
               exclude: Optional[Union[Tuple[torch.Tensor, torch.Tensor], Sequence[Sequence[int]]]] = None,
               kprime: Optional[int] = None, chunk_rows: Optional[int] = None,
               timer: Optional[_lib.Timer] = None, liked_counts: Optional[torch.Tensor] = None,
               liked_sum_hook=None, fuse: bool = True,
               t_floor_hook=None, theta_hook=None) -> "PendingTopk":
    """Enqueue the first pass of score_topk (see there) on the catalog's device and return
    without waiting for it: score_topk_finish(pending) waits, retries the queries whose
    certificate needs it and returns (scores, rows). Submitting batch i+1 before finishing
    batch i keeps the GPU busy while the host checks certificates (bench.py's step loop).
    Top-k by cosine (mean cosine over liked rows) with exclusions.

    Returns (scores float64 [B, k], rows int64 [B, k]) on the catalog's device, ordered by
    (score desc, row asc); rows are GLOBAL row ids; missing entries (fewer than k candidates)
    are NaN / -1. ``exclude`` and ``liked`` take device CSR pairs or host lists of global rows.

    t_floor_hook (row-sharded catalogs): hook(vals f32 [B, k], eps f32 [B]) -> float64 [B], a
    lower bound of the k-th best EXACT score over the whole catalog. vals are this shard's k
    best approx scores (-inf padded); every vals[b, j] - eps[b] bounds a distinct row's exact
    score from below, so the k-th largest of those bounds over all shards (union_floor, after
    an all-gather) is such a bound. The first pass then screens (ebt_cosine_screen), calls the
    hook, and rescores only the rows that can enter the GLOBAL top k (ebt_rescore with
    t_floor); slots that cut empties read NaN / -1, which merge_topk sorts last. The hook runs
    exactly once per call on every shard (retries below are local, no collective), so shards
    cannot fall out of step.

    Either hook may return a callable instead (a future: its collective was started
    asynchronously); it is called when the value is needed -- the next stage of
    score_topk_stages.

    theta_hook (with t_floor_hook): hook(qb, kprime) -> (theta f32 [B_pad], hits) or None, a
    catalog-wide screening threshold (distributed.py: the all-gathered sample maxima of every
    shard). Called exactly once per call, before the screen; when it returns a threshold and
    the fused wave-merge screen applies (k' <= 512), the shard is screened at theta
    (ebt_cosine_screen_at) and a query whose theta exceeds t_floor - eps is rerun unfused.
    """
    if t_floor_hook is None and theta_hook is None and liked_sum_hook is None and \
            liked_counts is None:
        # one catalog (or a shard queried on its own): the C ABI's self-contained path
        return _submit_c(catalog, k, queries, liked, exclude, kprime, chunk_rows, timer, fuse)
    g = score_topk_stages(catalog, k, queries=queries, liked=liked, exclude=exclude,
                          kprime=kprime, chunk_rows=chunk_rows, timer=timer,
                          liked_counts=liked_counts, liked_sum_hook=liked_sum_hook, fuse=fuse,
                          t_floor_hook=t_floor_hook, theta_hook=theta_hook)
    next(g)
    next(g)
    return next(g)


@dataclass
class PendingTopkC:
    """A batch submitted through ebt_cosine_topk_submit (the C ABI's self-contained path): the
    ebt_pending record plus every buffer it points at, kept alive until the finish."""
    pending: "_lib.EbtPending"
    catalog: Catalog
    opt: "_lib.EbtOptions"
    out_s: torch.Tensor
    out_r: torch.Tensor
    ws: torch.Tensor
    cert_host: torch.Tensor
    keep: tuple


_SKLEARN_EMPTY = "Found array with 0 sample(s)"


def _submit_c(catalog: Catalog, k: int, queries, liked, exclude, kprime, chunk_rows, timer,
              fuse) -> PendingTopkC:
    """score_topk_submit over ebt_cosine_topk_submit: query prep, the screen, the certificate
    and every retry run inside libebert (include/ebert.h); Python only owns the buffers."""
    import ctypes
    if k < 1:
        raise EbertError("k must be >= 1")
    dev = catalog.device
    if (queries is None) == (liked is None):
        raise EbertError("pass exactly one of queries= or liked=")
    if exclude is not None:
        exclude = (csr_from_lists(exclude, dev) if not isinstance(exclude, tuple)
                   else exclude if isinstance(exclude, SortedCSR) else csr_sorted(*exclude))
    q_ptr, q_dt, ldq, lo, lr, lo_csr = None, 0, 0, None, None, None
    if queries is not None:
        require_cuda(queries, "queries")
        if queries.dim() != 2 or queries.shape[1] != catalog.d:
            raise EbertError(f"queries must be [B, {catalog.d}], got {tuple(queries.shape)}")
        if queries.dtype not in DTYPE_CODE:
            raise EbertError(f"unsupported query dtype {queries.dtype}")
        if queries.stride(1) != 1:
            queries = queries.contiguous()
        B = int(queries.shape[0])
        q_ptr, q_dt, ldq = ptr(queries), DTYPE_CODE[queries.dtype], int(queries.stride(0))
    else:
        lo_csr = liked if isinstance(liked, tuple) else csr_from_lists(liked, dev)
        lo, lr = lo_csr
        B = int(lo.numel()) - 1
    if B < 1:
        raise EbertError("empty query batch")
    flags = 0 if fuse else _lib.EBT_FLAG_NO_FUSE
    if liked is not None and isinstance(lo_csr, SortedCSR) and lo_csr.checked_for(
            catalog.row_offset, catalog.row_offset + catalog.n):
        # checked on the host while building it: the C entry reads nothing back (no stream sync)
        flags |= _lib.EBT_FLAG_LIKED_CHECKED
    opt = _lib.EbtOptions(kprime=int(kprime or 0), flags=flags, chunk_rows=int(chunk_rows or 0))
    lib = _lib.load()
    need = lib.ebt_workspace_bytes(ctypes.byref(catalog.cstruct), B, k, ctypes.byref(opt))
    if need == 0:
        raise EbertError(f"k={k}, batch {B} over a {catalog.n}-row catalog is not supported "
                         f"(ebt_workspace_bytes returned 0)")
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    cert_host = torch.empty(B + 1, dtype=torch.int32, pin_memory=True)
    pend = _lib.EbtPending()
    eo, er = exclude if exclude is not None else (None, None)
    try:
        call("ebt_cosine_topk_submit", ctypes.byref(catalog.cstruct), q_ptr, q_dt, B, ldq,
             ptr(lo), ptr(lr), k, ptr(eo), ptr(er), ctypes.byref(opt), ptr(ws), need,
             ptr(out_s), ptr(out_r), ptr(cert_host), ctypes.byref(pend),
             timer.handle if timer is not None else None, stream_of(dev))
    except EbertError as e:
        msg = str(e)
        if _SKLEARN_EMPTY in msg:   # lib.py:51 on a user without liked movies (sklearn)
            raise ValueError(msg[msg.index(_SKLEARN_EMPTY):]) from None
        raise
    return PendingTopkC(pend, catalog, opt, out_s, out_r, ws, cert_host,
                        (queries, lo, lr, eo, er))


def score_topk_stages(catalog: Catalog, k: int, queries: Optional[torch.Tensor] = None,
                      liked=None, exclude=None, kprime: Optional[int] = None,
                      chunk_rows: Optional[int] = None, timer: Optional[_lib.Timer] = None,
                      liked_counts: Optional[torch.Tensor] = None, liked_sum_hook=None,
                      fuse: bool = True, t_floor_hook=None, theta_hook=None):
    """score_topk_submit as a generator of three stages, so a caller can interleave the stages
    of consecutive batches (distributed.py: each stage of a row-sharded batch ends in a
    collective, and the next stage of the OTHER batch runs while it is in flight):
      next() #1: query prep and theta_hook (the shared threshold's all-gather);
      next() #2: the screen and t_floor_hook (the floor's all-gather);
      next() #3: the rescore; returns the PendingTopk (score_topk_finish completes it).
    Without t_floor_hook the whole first pass runs in stage 2."""
    if k < 1:
        raise EbertError("k must be >= 1")
    dev = catalog.device
    if liked is not None and not isinstance(liked, tuple):
        liked = csr_from_lists(liked, dev)
    if exclude is not None:
        exclude = (csr_from_lists(exclude, dev) if not isinstance(exclude, tuple)
                   else exclude if isinstance(exclude, SortedCSR) else csr_sorted(*exclude))
    if theta_hook is not None and t_floor_hook is None:
        raise EbertError("theta_hook needs t_floor_hook (the threshold is verified against it)")
    with region(timer, "prep", dev):
        qb = prepare_queries(catalog, queries=queries, liked=liked, liked_counts=liked_counts,
                             liked_sum_hook=liked_sum_hook)
    n_cap = _round_up(catalog.n, 4)
    k_eff = min(k, catalog.n)
    if k_eff > KPRIME_MAX:
        raise EbertError(f"k={k} > {KPRIME_MAX} over a {catalog.n}-row catalog is not supported")
    kp = kprime or default_kprime(catalog, k_eff)
    kp = max(_round_up(k_eff, 4), min(_round_up(kp, 4), n_cap, KPRIME_MAX))
    flags = 0 if fuse else _lib.EBT_FLAG_NO_FUSE
    t_floor = None
    if t_floor_hook is None:
        yield
        s, r, cert = run_pipeline(catalog, qb, k_eff, kp, exclude, chunk_rows, timer, flags=flags)
        yield
    else:
        cut = _global_cut_stages(catalog, qb, k_eff, k, kp, exclude, chunk_rows, timer, flags,
                                 t_floor_hook, theta_hook)
        next(cut)
        yield
        next(cut)
        yield
        s, r, cert, t_floor = next(cut)
    # the certificates travel to pinned host memory right behind this batch's kernels, so
    # finishing it waits for this batch only, not for batches submitted after it
    cert_host = torch.empty(cert.shape, dtype=cert.dtype, pin_memory=True)
    cert_host.copy_(cert, non_blocking=True)
    ready = torch.cuda.Event()
    ready.record(torch.cuda.current_stream(dev))
    yield PendingTopk(catalog, qb, k, k_eff, kp, exclude, chunk_rows, timer, flags, n_cap,
                      s, r, cert, cert_host, ready, t_floor)


def score_topk_finish(p) -> Tuple[torch.Tensor, torch.Tensor]:
    """Wait for a submitted batch, run its retries, return (scores f64 [B, k], rows i64 [B, k])."""
    if isinstance(p, PendingTopkC):
        import ctypes
        call("ebt_cosine_topk_finish", ctypes.byref(p.pending))
        return p.out_s, p.out_r
    catalog, qb, k, k_eff, kp = p.catalog, p.qb, p.k, p.k_eff, p.kprime
    exclude, chunk_rows, timer, flags, n_cap = p.exclude, p.chunk_rows, p.timer, p.flags, p.n_cap
    s, r, cert = p.s, p.r, p.cert
    dev = catalog.device
    p.ready.synchronize()
    flat = p.cert_host
    # retries, only for the queries that need one: a fused candidate list that overflowed
    # (cert -1: rerun unfused) or a candidate set that is not provably complete (cert 0: widen k')
    while True:
        if flat is None:
            flat = cert.cpu()
        if bool((flat == -3).any()):   # the rescore's check of the exclusion segments
            raise EbertError("exclusion rows must be sorted ascending within each query")
        if bool((flat == -2).any()):
            raise EbertError("internal error: candidate row out of range (libebert bug)")
        over = torch.nonzero(flat == -1).flatten().to(dev)
        bad = torch.nonzero(flat == 0).flatten().to(dev)
        if over.numel() == 0 and bad.numel() == 0:
            break
        flat = None
        if over.numel():
            sub_ex = csr_subset(exclude[0], exclude[1], over) if exclude is not None else None
            s2, r2, c2 = run_pipeline(catalog, qb.subset(over), k_eff, kp, sub_ex, chunk_rows,
                                      timer, flags=_lib.EBT_FLAG_NO_FUSE)
            s[over], r[over], cert[over] = s2, r2, c2
            continue
        widen = kp < min(n_cap, KPRIME_MAX)
        if not widen and flags & _lib.EBT_FLAG_EXACT:
            raise EbertError(f"{bad.numel()} queries could not be certified at k'={kp} "
                             "(more than k' rows tie with the k-th score at f32 precision)")
        if widen:
            kp = min(kp * 4, n_cap, KPRIME_MAX)
        else:
            # the f16/bf16 screen's error bound spans more than k' = 4096 rows around the
            # k-th score: screen these queries again in float64 (EBT_FLAG_EXACT), from the
            # default k' up
            flags = _lib.EBT_FLAG_EXACT
            kp = max(_round_up(k_eff, 4), min(_round_up(default_kprime(catalog, k_eff), 4),
                                              n_cap, KPRIME_MAX))
        sub_ex = csr_subset(exclude[0], exclude[1], bad) if exclude is not None else None
        s2, r2, c2 = run_pipeline(catalog, qb.subset(bad), k_eff, kp, sub_ex, chunk_rows, timer,
                                  flags=flags)
        s[bad], r[bad], cert[bad] = s2, r2, c2
    if k_eff < k:
        pad_s = torch.full((qb.B, k - k_eff), float("nan"), dtype=torch.float64, device=dev)
        pad_r = torch.full((qb.B, k - k_eff), -1, dtype=torch.int64, device=dev)
        s, r = torch.cat([s, pad_s], 1), torch.cat([r, pad_r], 1)
    return s, r


def score_topk(catalog: Catalog, k: int, queries: Optional[torch.Tensor] = None,
               liked: Optional[Union[Tuple[torch.Tensor, torch.Tensor], Sequence[Sequence[int]]]] = None,
               exclude: Optional[Union[Tuple[torch.Tensor, torch.Tensor], Sequence[Sequence[int]]]] = None,
               kprime: Optional[int] = None, chunk_rows: Optional[int] = None,
               timer: Optional[_lib.Timer] = None, liked_counts: Optional[torch.Tensor] = None,
               liked_sum_hook=None, fuse: bool = True,
               t_floor_hook=None, theta_hook=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k by cosine (mean cosine over liked rows) with exclusions: score_topk_submit +
    score_topk_finish (arguments and results as documented there)."""
    return score_topk_finish(score_topk_submit(
        catalog, k, queries=queries, liked=liked, exclude=exclude, kprime=kprime,
        chunk_rows=chunk_rows, timer=timer, liked_counts=liked_counts,
        liked_sum_hook=liked_sum_hook, fuse=fuse, t_floor_hook=t_floor_hook,
        theta_hook=theta_hook))


@dataclass
class PendingTopk:
    """A submitted score_topk batch: its first pass is enqueued, retries not yet decided."""
    catalog: Catalog
    qb: QueryBatch
    k: int
    k_eff: int
    kprime: int
    exclude: Optional[Tuple[torch.Tensor, torch.Tensor]]
    chunk_rows: Optional[int]
    timer: Optional[_lib.Timer]
    flags: int
    n_cap: int
    s: torch.Tensor
    r: torch.Tensor
    cert: torch.Tensor
    cert_host: torch.Tensor          # pinned copy of cert, valid once `ready` has completed
    ready: torch.cuda.Event
    t_floor: Optional[torch.Tensor] = None   # the catalog-wide floor (t_floor_hook), f64 [B]


def union_floor_gathered(g: torch.Tensor, k: int) -> torch.Tensor:
    """ebt_union_floor over an all-gathered [R, B, k'+1] f32 tensor (the shards' k' best approx,
    then their eps): float64 [B]."""
    g = g.contiguous()
    R, B, ld = g.shape
    out = torch.empty(B, dtype=torch.float64, device=g.device)
    call("ebt_union_floor", ptr(g), R, B, ld, k, ptr(out), stream_of(g.device))
    return out


def union_floor(vals: torch.Tensor, eps: torch.Tensor, k: int) -> torch.Tensor:
    """The k-th largest of vals[r, b, j] - eps[r, b] over all shards r and slots j: a lower bound
    of query b's k-th best exact score (vals f32 [R, B, k] approx, eps f32 [R, B]); one
    ebt_union_floor launch on the device (no CPU path: CPU tensors raise EbertError)."""
    require_cuda(vals, "union_floor vals")
    g = torch.cat([vals.float(), eps.float()[:, :, None]], 2).contiguous()
    return union_floor_gathered(g, k)


def _screen_global_cut(catalog: Catalog, qb: QueryBatch, k: int, k_req: int, kprime: int,
                       exclude, chunk_rows, timer, flags, t_floor_hook, theta_hook=None):
    """score_topk's first pass under a catalog-wide cut: [theta_hook,] screen, t_floor_hook,
    rescore. A shard with fewer rows than the requested k_req pads its bounds with -inf."""
    g = _global_cut_stages(catalog, qb, k, k_req, kprime, exclude, chunk_rows, timer, flags,
                           t_floor_hook, theta_hook)
    next(g)
    next(g)
    return next(g)[:3]


def _global_cut_stages(catalog: Catalog, qb: QueryBatch, k: int, k_req: int, kprime: int,
                       exclude, chunk_rows, timer, flags, t_floor_hook, theta_hook=None):
    """_screen_global_cut as a generator: yields after the theta hook and after the floor hook,
    then yields (scores, rows, cert, t_floor)."""
    dev = catalog.device
    B = qb.B
    # the hook is a collective: called on every shard whether or not this one uses its result
    th = theta_hook(qb, kprime) if theta_hook is not None else None
    yield
    if callable(th):  # a future: the hook's collective was started, its result is needed now
        th = th()
    use_theta = th is not None and flags == 0 and kprime <= MERGE_WAVE_KMAX
    if use_theta:
        lv, lr, ovf, eps = screen_at(catalog, qb, k, kprime, th[0], th[1], exclude, chunk_rows,
                                     timer)
    else:
        lv, lr, ovf, eps = run_screen(catalog, qb, k, kprime, exclude, chunk_rows, timer, flags)
    vals = lv[:, :k]
    if k < k_req:
        vals = torch.cat([vals, torch.full((B, k_req - k), float("-inf"), device=dev)], 1)
    t_floor = t_floor_hook(vals.contiguous(), eps[:B].contiguous())
    yield
    if callable(t_floor):
        t_floor = t_floor()
    t_floor = t_floor.contiguous()
    if t_floor.dtype != torch.float64 or t_floor.shape != (B,):
        raise EbertError("t_floor_hook must return float64 [B]")
    local = lr - catalog.row_offset if catalog.row_offset else lr
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    cert = torch.empty(B, dtype=torch.int32, device=dev)
    call("ebt_rescore", ptr(qb.q64), B, catalog.d, ptr(catalog.data), catalog.dtype_code,
         catalog.ld, ptr(catalog.gnorm), catalog.row_offset, ptr(lv), ptr(local.contiguous()),
         kprime, k, catalog.n, ptr(eps), ptr(t_floor), ptr(out_s), ptr(out_r), ptr(cert),
         timer.handle if timer is not None else None, stream_of(dev))
    # an overflowed fused list is rerun unfused (cert -1), unless a row is corrupt (-2); so is a
    # query whose shared threshold may have dropped a row of the global top k: every top-k row
    # has approx >= t_floor - eps, so theta <= t_floor - eps keeps them all
    with region(timer, "small", dev):
        call("ebt_certify_cut", ptr(cert), ptr(ovf), ptr(th[0]) if use_theta else None,
             ptr(t_floor), ptr(eps), B, stream_of(dev))
    yield out_s, out_r, cert, t_floor


def merge_topk(scores: torch.Tensor, rows: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge [R, B, k] partial lists (the all-gathered shard results) into the global top-k."""
    require_cuda(scores, "scores")
    R, B, kk = scores.shape
    scores = scores.contiguous()
    rows = rows.contiguous()
    out_s = torch.empty((B, k), dtype=torch.float64, device=scores.device)
    out_r = torch.empty((B, k), dtype=torch.int64, device=scores.device)
    if kk != k:
        raise EbertError("partial lists must have k entries")
    call("ebt_merge_topk", ptr(scores), ptr(rows), R, B, k, ptr(out_s), ptr(out_r),
         stream_of(scores.device))
    return out_s, out_r


def rescore_rows(catalog: Catalog, qb: QueryBatch, cand_rows: torch.Tensor
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact float64 cosine of each query against its OWN candidate rows ([B, m] global rows),
    sorted (score desc, row asc). This is lib.py:105-106 (mean cosine of the liked movies vs the
    query matches) when qb holds the liked-row means."""
    dev = catalog.device
    B, m = cand_rows.shape
    local = (cand_rows - catalog.row_offset).contiguous()
    vals = torch.zeros((B, m), dtype=torch.float32, device=dev)
    eps = torch.zeros(max(B, 1), dtype=torch.float32, device=dev)
    out_s = torch.empty((B, m), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, m), dtype=torch.int64, device=dev)
    cert = torch.empty(B, dtype=torch.int32, device=dev)
    call("ebt_rescore", ptr(qb.q64), B, catalog.d, ptr(catalog.data), catalog.dtype_code,
         catalog.ld, ptr(catalog.gnorm), catalog.row_offset, ptr(vals), ptr(local), m, m, catalog.n,
         ptr(eps), None, ptr(out_s), ptr(out_r), ptr(cert), None, stream_of(dev))
    return out_s, out_r
