"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

This module is the float64 restatement of the reference's recommend/top-K hot path. Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker (or as the timed CPU baseline). The product package ``robot_ebert_amd``
never imports it and has no CPU fallback.

Pinning: ``tests/golden/make_golden.py`` imported the reference's own ``get_user_recs``
(``/root/reference/src/backend/app/lib.py``) with its network/database clients stubbed, ran it
on seeded synthetic catalogs, and committed the outputs under ``tests/golden/``.
``tests/test_oracle_golden.py`` checks this restatement against those vectors, and against
scikit-learn's ``cosine_similarity`` + a pandas sort (the third-party code the reference calls).

Reference call chain being restated (file:line into /root/reference):
  * ``src/backend/app/lib.py:32-63``  get_user_recs
      - ``:36-40``  ratings fetch, empty -> ``[]``
      - ``:43-48``  keep ratings whose tmdb_id is in the catalog; liked = rating >= 3.5
                    (``constants.py:19``); candidates = catalog.index.difference(rated)
      - ``:51``     cosine_similarity(catalog.loc[liked], catalog)
      - ``:52``     .mean(axis=0)
      - ``:55``     .loc[unrated].sort_values(ascending=False)[:k].sort_index()
      - ``:58-63``  hydrate + zip + stable sort by score desc
  * scikit-learn ``metrics/pairwise.py:1683-1738`` (cosine_similarity),
    ``preprocessing/_data.py:2011-2015`` (normalize) and ``:118-123`` (_handle_zeros_in_scale:
    a row norm < 10*eps is replaced by 1).
  * ``lib.py:105-106,117`` run_search re-weighting (mean cosine over the query matches and
    ``0.9*query + 0.1*user``, ``constants.py:20``).

Ordering: the reference's descending sort is numpy introsort (unstable, pandas
``core/sorting.py:436-441``). This restatement and the GPU path both define the order as
(score desc, row asc); parity inputs are continuous Gaussians so exact ties have probability 0.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

EPS64 = np.finfo(np.float64).eps
LIKED_MOVIE_SCORE = 3.5  # constants.py:19
QUERY_SCORE_WEIGHT = 0.90  # constants.py:20


def zero_guard_norms(norms: np.ndarray) -> np.ndarray:
    """sklearn ``_handle_zeros_in_scale`` (preprocessing/_data.py:118-123): norm < 10*eps -> 1."""
    norms = np.array(norms, dtype=np.float64, copy=True)
    norms[norms < 10 * EPS64] = 1.0
    return norms


def row_norms(x: np.ndarray) -> np.ndarray:
    """sklearn ``row_norms`` (utils/extmath.py:76): sqrt(einsum('ij,ij->i'))."""
    x = np.asarray(x, dtype=np.float64)
    return np.sqrt(np.einsum("ij,ij->i", x, x))


def normalize_rows(x: np.ndarray) -> np.ndarray:
    """sklearn ``normalize(norm='l2')`` (preprocessing/_data.py:2011-2015), float64."""
    x = np.asarray(x, dtype=np.float64)
    return x / zero_guard_norms(row_norms(x))[:, None]


def cosine_similarity(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """sklearn ``cosine_similarity`` restated in float64 (metrics/pairwise.py:1683-1738).

    Raises the same ValueError as ``check_pairwise_arrays`` for an empty X.
    """
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if x.shape[0] == 0:
        raise ValueError(
            f"Found array with 0 sample(s) (shape={x.shape}) while a minimum of 1 is required "
            "by check_pairwise_arrays."
        )
    return normalize_rows(x) @ normalize_rows(y).T


def mean_cosine_query(liked_rows: np.ndarray) -> np.ndarray:
    """q = mean_i normalize(liked_i), NOT re-normalised (lib.py:51-52 folded into the query)."""
    return normalize_rows(liked_rows).mean(axis=0)


def order_desc(scores: np.ndarray, rows: np.ndarray) -> np.ndarray:
    """Permutation sorting by (score desc, row asc)."""
    return np.lexsort((rows, -scores))


def topk_from_scores(scores: np.ndarray, k: int, exclude: Optional[Iterable[int]] = None
                     ) -> Tuple[np.ndarray, np.ndarray]:
    """Top-k of one score row after removing excluded rows (lib.py:55), order (score desc, row asc).

    Returns (scores f64 [m], rows i64 [m]) with m = min(k, #candidates).
    """
    scores = np.asarray(scores, dtype=np.float64)
    rows = np.arange(scores.shape[0], dtype=np.int64)
    if exclude is not None:
        mask = np.ones(scores.shape[0], dtype=bool)
        ex = np.asarray(list(exclude), dtype=np.int64)
        if ex.size:
            mask[ex] = False
        rows = rows[mask]
        scores = scores[mask]
    if k < rows.shape[0]:
        # partition first (fast), then exact order on a widened boundary
        kk = min(rows.shape[0], k + 64)
        part = np.argpartition(-scores, kk - 1)[:kk]
        # widen so every value tied with the kk-th is included
        thr = scores[part].min()
        part = np.nonzero(scores >= thr)[0]
        rows, scores = rows[part], scores[part]
    order = order_desc(scores, rows)[:k]
    return scores[order], rows[order]


def cosine_topk(queries: np.ndarray, catalog: np.ndarray, k: int,
                exclude: Optional[Sequence[Iterable[int]]] = None,
                chunk: int = 64) -> Tuple[np.ndarray, np.ndarray]:
    """Batched single-vector queries (L=1): float64 cosine + per-query top-k.

    Returns padded arrays (scores f64 [B,k] NaN-padded, rows i64 [B,k] -1-padded).
    """
    queries = np.asarray(queries, dtype=np.float64)
    catalog = np.asarray(catalog, dtype=np.float64)
    cn = normalize_rows(catalog)
    B = queries.shape[0]
    out_s = np.full((B, k), np.nan)
    out_r = np.full((B, k), -1, dtype=np.int64)
    for b0 in range(0, B, chunk):
        qn = normalize_rows(queries[b0:b0 + chunk])
        s = qn @ cn.T
        for i in range(s.shape[0]):
            ex = None if exclude is None else exclude[b0 + i]
            sc, rw = topk_from_scores(s[i], k, ex)
            out_s[b0 + i, :sc.shape[0]] = sc
            out_r[b0 + i, :rw.shape[0]] = rw
    return out_s, out_r


def _chunk_topk(qn: np.ndarray, row0: int, chunk: np.ndarray, k: int,
                exclude: Optional[Sequence[np.ndarray]]) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Per-query top-k (ties at the cut kept) of one catalog row block, float64."""
    c = np.asarray(chunk, dtype=np.float64)
    s = (qn @ c.T) / zero_guard_norms(row_norms(c))[None, :]   # == normalize(q) . normalize(c)
    out = []
    for i in range(s.shape[0]):
        ex = None
        if exclude is not None:
            e = exclude[i]
            e = e[(e >= row0) & (e < row0 + c.shape[0])] - row0
            ex = e
        sc, rw = topk_from_scores(s[i], k, ex)
        # topk_from_scores cuts at exactly k; keep every value tied with the k-th as well, so a
        # later merge still orders equal scores by row
        if sc.shape[0] == k:
            row = s[i].copy()
            if ex is not None and len(ex):
                row[ex] = -np.inf
            tied = np.nonzero(row == sc[-1])[0]
            extra = np.setdiff1d(tied, rw, assume_unique=False)
            if extra.size:
                sc = np.concatenate([sc, row[extra]])
                rw = np.concatenate([rw, extra])
        out.append((sc, rw + row0))
    return out


def cosine_topk_stream(queries: np.ndarray, chunks: Iterable[Tuple[int, np.ndarray]], k: int,
                       exclude: Optional[Sequence[Iterable[int]]] = None, workers: int = 8
                       ) -> Tuple[np.ndarray, np.ndarray]:
    """``cosine_topk`` over a catalog delivered as row blocks ``(row0, rows[r, d])``.

    Same arithmetic as ``cosine_topk`` (lib.py:51 via sklearn normalise + dot, float64; lib.py:55
    exclusion + (score desc, row asc) top-k), but it never holds the catalog in float64: each
    block is upcast, scored and reduced to its per-query top-k (all values tied with the k-th
    kept), and the blocks' lists are merged at the end. This is what lets the tests check the
    BASELINE workloads (up to 10M x 768 and 6.25M x 1536 per GPU) against the host oracle.
    Blocks are processed by ``workers`` threads (numpy releases the GIL in upcasts and GEMMs).
    """
    from concurrent.futures import ThreadPoolExecutor

    qn = normalize_rows(np.asarray(queries, dtype=np.float64))
    B = qn.shape[0]
    ex = None
    if exclude is not None:
        ex = [np.asarray(sorted(set(int(v) for v in e)), dtype=np.int64) for e in exclude]
    parts: List[List[Tuple[np.ndarray, np.ndarray]]] = []
    workers = max(1, workers)
    with ThreadPoolExecutor(max_workers=workers) as pool:
        pending = []
        for r0, blk in chunks:   # at most 2 x workers blocks in host memory at once
            pending.append(pool.submit(_chunk_topk, qn, int(r0), blk, k, ex))
            if len(pending) >= 2 * workers:
                parts.append(pending.pop(0).result())
        parts.extend(f.result() for f in pending)
    out_s = np.full((B, k), np.nan)
    out_r = np.full((B, k), -1, dtype=np.int64)
    for b in range(B):
        if not parts:
            break
        s = np.concatenate([p[b][0] for p in parts])
        r = np.concatenate([p[b][1] for p in parts])
        o = order_desc(s, r)[:k]
        out_s[b, :o.shape[0]] = s[o]
        out_r[b, :o.shape[0]] = r[o]
    return out_s, out_r


def liked_topk(catalog: np.ndarray, liked: Sequence[Sequence[int]], k: int,
               exclude: Optional[Sequence[Iterable[int]]] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Mean-over-liked cosine (lib.py:51-52) + exclusion + top-k (lib.py:55), per user."""
    catalog = np.asarray(catalog, dtype=np.float64)
    B = len(liked)
    out_s = np.full((B, k), np.nan)
    out_r = np.full((B, k), -1, dtype=np.int64)
    for b in range(B):
        rows = np.asarray(liked[b], dtype=np.int64)
        s = cosine_similarity(catalog[rows], catalog).mean(axis=0)  # raises for L == 0
        ex = None if exclude is None else exclude[b]
        sc, rw = topk_from_scores(s, k, ex)
        out_s[b, :sc.shape[0]] = sc
        out_r[b, :rw.shape[0]] = rw
    return out_s, out_r


def get_user_recs(ratings: Sequence[Tuple[str, float]], catalog_ids: Sequence[str],
                  catalog: np.ndarray, k: int = 10,
                  liked_threshold: float = LIKED_MOVIE_SCORE) -> List[Tuple[str, float]]:
    """Restatement of lib.py:32-63 on in-memory data.

    ``ratings`` is the user's (tmdb_id, rating) list (the SQL result of lib.py:36-38).
    Returns [(tmdb_id, score)] in the reference's final order: the top-k chosen by score desc,
    re-sorted by string id (lib.py:55 ``sort_index``), then stable-sorted by score desc
    (lib.py:63). Raises ValueError for a user with ratings but no liked movie in the catalog.
    """
    if not ratings:  # lib.py:39-40
        return []
    ids = list(catalog_ids)
    pos = {t: i for i, t in enumerate(ids)}
    kept = [(t, r) for (t, r) in ratings if t in pos]  # lib.py:44
    liked = [pos[t] for (t, r) in kept if r >= liked_threshold]  # lib.py:47
    rated = {pos[t] for (t, _) in kept}  # lib.py:48 (all ratings, any value)
    catalog = np.asarray(catalog, dtype=np.float64)
    sims = cosine_similarity(catalog[np.asarray(liked, dtype=np.int64)], catalog)  # lib.py:51
    scores = sims.mean(axis=0)  # lib.py:52
    sc, rw = topk_from_scores(scores, k, sorted(rated))  # lib.py:55 (sort + [:k])
    picked = sorted(zip((ids[r] for r in rw), sc), key=lambda t: t[0])  # .sort_index()
    return sorted(picked, key=lambda t: t[1], reverse=True)  # lib.py:63 (stable)


def reweight_scores(query_scores: np.ndarray, user_scores: np.ndarray,
                    weight: float = QUERY_SCORE_WEIGHT) -> np.ndarray:
    """lib.py:117: weight*query + (1-weight)*user."""
    return weight * np.asarray(query_scores, np.float64) + (1 - weight) * np.asarray(user_scores, np.float64)


def merge_topk(scores: np.ndarray, rows: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Merge R partial top-k lists per query ([R,B,k] each) into the global top-k."""
    R, B, _ = scores.shape
    out_s = np.full((B, k), np.nan)
    out_r = np.full((B, k), -1, dtype=np.int64)
    for b in range(B):
        s = scores[:, b, :].reshape(-1)
        r = rows[:, b, :].reshape(-1)
        m = r >= 0
        s, r = s[m], r[m]
        o = order_desc(s, r)[:k]
        out_s[b, :o.shape[0]] = s[o]
        out_r[b, :o.shape[0]] = r[o]
    return out_s, out_r
