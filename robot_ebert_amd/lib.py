"""Drop-in GPU version of the reference's recommend call surface (src/backend/app/lib.py).

``get_user_recs(user_id, k)`` keeps ``lib.py:32-63``'s Python semantics -- the same SQL, the same
pandas filtering, the same ValueError for a user without liked movies, the same
``sort_index``/``zip``/``sorted`` hydration order -- and replaces only the scoring block
``lib.py:51-55`` (sklearn cosine_similarity + mean + pandas sort) by ``search.score_topk`` on the
HBM-resident catalog. ``user_movie_scores`` mirrors the re-weighting arithmetic of
``lib.py:94-121`` for ``run_search`` (whose LLM / Chroma retrieval is out of scope).

Module globals play the role of ``backend.app.constants`` (engine, catalog, thresholds) and are
set with ``configure``.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch
from sqlalchemy import select

from . import tables
from .catalog import Catalog
from .models import Movie, Recommendation
from .search import csr_from_lists, prepare_queries, rescore_rows, score_topk

LIKED_MOVIE_SCORE = 3.5   # constants.py:19
QUERY_SCORE_WEIGHT = 0.90  # constants.py:20
SIMILARITY_TOP_K = 10     # constants.py:21

engine = None                              # constants.py:26 (caller-supplied SQLAlchemy Engine)
movies_collab_catalog: Optional[Catalog] = None  # constants.py:55-56, resident in HBM
movies_content_catalog: Optional[Catalog] = None  # the movies-content collection (constants.py:29-53)
_get_movies_override: Optional[Callable[[List[str]], List[Movie]]] = None


def configure(engine=None, catalog: Optional[Catalog] = None,
              get_movies: Optional[Callable[[List[str]], List[Movie]]] = None,
              content_catalog: Optional[Catalog] = None) -> None:
    """Install the process-global resources (the reference builds them at import time)."""
    g = globals()
    if engine is not None:
        g["engine"] = engine
    if catalog is not None:
        g["movies_collab_catalog"] = catalog
    if content_catalog is not None:
        g["movies_content_catalog"] = content_catalog
    g["_get_movies_override"] = get_movies


def get_movies(tmdb_ids: List[str]) -> List[Movie]:
    """lib.py:23-29: Movie rows for the ids, ORDER BY tmdb_id."""
    if _get_movies_override is not None:
        return _get_movies_override(tmdb_ids)
    with engine.begin() as cnx:
        stmt = select(tables.movies).where(tables.movies.c.tmdb_id.in_(tmdb_ids)).order_by(
            tables.movies.c.tmdb_id)
        rows = cnx.execute(stmt).all()
    out = []
    for row in rows:
        d = row._asdict()
        d.pop("updated_at", None)
        out.append(Movie(**d))
    return out


def _user_ratings(user_id: str) -> pd.DataFrame:
    """lib.py:36-38 + 43-44: the user's ratings restricted to movies in the catalog."""
    with engine.begin() as cnx:
        rows = cnx.execute(select(tables.ratings).where(tables.ratings.c.user_id == user_id)).all()
    if not rows:  # pandas: an empty DataFrame has no "tmdb_id" column (lib.py:97)
        raise KeyError("tmdb_id")
    df = pd.DataFrame(rows)
    cat = movies_collab_catalog
    return df[cat.contains(df["tmdb_id"])]


def user_query_lists(user_ratings: pd.DataFrame, catalog: Catalog,
                     liked_threshold: float = LIKED_MOVIE_SCORE) -> Tuple[List[int], List[int]]:
    """lib.py:47-48 as row lists: (liked rows, rated rows). The reference's candidate set is
    catalog.index.difference(rated), i.e. every catalog row except the rated ones."""
    liked_ids = user_ratings[user_ratings["rating"] >= liked_threshold]["tmdb_id"]
    rated_ids = pd.unique(user_ratings["tmdb_id"])
    return catalog.rows_of(liked_ids), catalog.rows_of(rated_ids)


def order_recommendations(pairs: Sequence[Tuple[str, float]]) -> List[Tuple[str, float]]:
    """lib.py:55 ``.sort_index()`` (lexicographic on the string ids) -- the order in which
    lib.py:58-62 zips the movies with the scores -- then lib.py:63's stable sort by score."""
    by_id = sorted(pairs, key=lambda t: t[0])
    return sorted(by_id, key=lambda t: t[1], reverse=True)


def _user_request(user_id: str) -> Optional[Tuple[List[int], List[int]]]:
    """lib.py:36-48: (liked rows, rated rows) of a user, None when the user has no ratings;
    sklearn's ValueError when none of the ratings is a liked catalog movie."""
    cat = movies_collab_catalog
    with engine.begin() as cnx:  # lib.py:36-40
        statement = select(tables.ratings).where(tables.ratings.c.user_id == user_id)
        user_ratings = cnx.execute(statement).all()
        if not user_ratings:
            return None
    # lib.py:43-48 on the fetched rows in plain Python (the DataFrame construction and boolean
    # indexing cost ~2 ms of interpreter time per request, under FastAPI's 40 worker threads
    # all of it serialised on the GIL): keep the ratings of catalog movies (the isin of :44),
    # liked = ratings >= LIKED_MOVIE_SCORE in row order (:47), rated = their ids in first-seen
    # order (:48, pd.unique) -- the lists user_query_lists builds from the DataFrame.
    pos = cat.index_pos
    kept = [(r.tmdb_id, r.rating) for r in user_ratings if r.tmdb_id in pos]  # lib.py:44
    liked = cat.rows_of([t for t, rt in kept if rt >= LIKED_MOVIE_SCORE])     # lib.py:47
    rated = cat.rows_of(list(dict.fromkeys(t for t, _ in kept)))              # lib.py:48
    if not liked:  # sklearn check_pairwise_arrays on an empty X (lib.py:51)
        raise ValueError(f"Found array with 0 sample(s) (shape=(0, {cat.d})) while a minimum of 1 "
                         "is required by check_pairwise_arrays.")
    return liked, rated


def _hydrate(s: np.ndarray, r: np.ndarray) -> List[Recommendation]:
    """lib.py:55-63 after the top-k: ids, sort_index, get_movies (ORDER BY id), zip, stable sort."""
    cat = movies_collab_catalog
    pairs = [(cat.id_of(int(rr)), float(ss)) for ss, rr in zip(s, r) if rr >= 0]
    ordered_by_id = sorted(pairs, key=lambda t: t[0])  # .sort_index()
    movies = get_movies(tmdb_ids=[t for t, _ in ordered_by_id])  # lib.py:58
    scores_by_id = [sc for _, sc in ordered_by_id]  # lib.py:59
    recommendations = [Recommendation(movie=m, score=sc) for m, sc in zip(movies, scores_by_id)]
    return sorted(recommendations, key=lambda x: x.score, reverse=True)  # lib.py:63


def get_user_recs(user_id: str, k: int = 10) -> List[Recommendation]:
    """GPU drop-in for lib.py:32-63 (same inputs, same outputs, same errors).

    Any k, as the reference's pandas `[:k]` (min(k, rows) > 4096 runs the full-sort path of
    csrc/large_k.hip). On a row-sharded catalog min(k, rows) <= 4096."""
    req = _user_request(user_id)
    if req is None:
        return []
    liked, rated = req
    scores, rows = score_topk(movies_collab_catalog, k, liked=[liked], exclude=[rated])  # :51-55
    return _hydrate(scores[0].cpu().numpy(), rows[0].cpu().numpy())


get_user_recs_gpu = get_user_recs  # SURVEY §8b's name for the drop-in


def get_user_recs_batched(batcher, user_id: str, k: int = 10) -> List[Recommendation]:
    """``get_user_recs`` whose scoring step is coalesced with concurrent callers by a
    ``batcher.RecBatcher`` over ``movies_collab_catalog``: same SQL, same errors,
    same ordering; the GPU sees one batch for many request threads."""
    req = _user_request(user_id)
    if req is None:
        return []
    liked, rated = req
    s, r = batcher.submit(liked, rated, k).result()
    return _hydrate(s, r)


def retrieve_content_matches(query_embedding, k: int = SIMILARITY_TOP_K) -> Tuple[List[str],
                                                                                   List[float]]:
    """the content retrieval of run_search (lib.py:71-73: the chat engine's
    ``similarity_top_k`` matches from the ``movies-content`` Chroma collection, hnsw:space=cosine,
    constants.py:29-53) as EXACT cosine top-k on the HBM content catalog. Returns (ids, cosine
    scores) in score order. HNSW is approximate; its result sets are not pinned."""
    cat = movies_content_catalog
    q = torch.as_tensor(np.asarray(query_embedding, dtype=np.float64).reshape(1, -1),
                        device=cat.device)
    scores, rows = score_topk(cat, k, queries=q)
    s, r = scores[0].cpu().numpy(), rows[0].cpu().numpy()
    keep = r >= 0
    return [cat.id_of(int(x)) for x in r[keep]], [float(x) for x in s[keep]]


def run_search_exact(query_embedding, user_id: Optional[str] = None,
                     k: int = SIMILARITY_TOP_K) -> List[Recommendation]:
    """lib.py:66-122 without the LLM: exact content retrieval of the query embedding, then the
    reference's re-ranking (user mean-cosine or popularity, 0.9 / 0.1 weights)."""
    ids, scores = retrieve_content_matches(query_embedding, k)
    return rerank_search_matches(ids, scores, user_id)


def user_movie_scores(user_id: str, match_ids: List[str]) -> pd.Series:
    """lib.py:94-106: mean cosine of the user's liked movies vs the query matches, float64,
    indexed by the match ids (in the given order). Raises ValueError when the user has no liked
    movie, exactly like the reference (its no-liked branch at :101-102 falls through into
    cosine_similarity with 0 rows)."""
    cat = movies_collab_catalog
    ur = _user_ratings(user_id)
    liked = cat.rows_of(ur[ur["rating"] >= LIKED_MOVIE_SCORE]["tmdb_id"])
    if not liked:
        raise ValueError(f"Found array with 0 sample(s) (shape=(0, {cat.d})) while a minimum of 1 "
                         "is required by check_pairwise_arrays.")
    qb = prepare_queries(cat, liked=csr_from_lists([liked], cat.device))
    match_rows = torch.tensor([cat.rows_of(match_ids)], dtype=torch.int64, device=cat.device)
    s, r = rescore_rows(cat, qb, match_rows)
    by_row = dict(zip(r[0].cpu().tolist(), s[0].cpu().tolist()))
    rows = cat.rows_of(match_ids)
    return pd.Series([by_row[x] for x in rows], index=list(match_ids))


def reweight(query_movie_scores: pd.Series, user_scores: pd.Series,
             weight: float = QUERY_SCORE_WEIGHT) -> pd.Series:
    """lib.py:117: weighted average of the query and user scores, sorted by id."""
    return (weight * query_movie_scores + (1 - weight) * user_scores).sort_index()


def popularity_scores(movies: List[Movie]) -> pd.Series:
    """lib.py:111-114: min-max scaled popularity of the query matches (no user given)."""
    s = pd.Series(data=[m.popularity for m in movies], index=[m.tmdb_id for m in movies])
    return (s - s.min()) / (s.max() - s.min())


def rerank_search_matches(match_ids: List[str], match_scores: List[float],
                          user_id: Optional[str] = None) -> List[Recommendation]:
    """lib.py:81-122 after the chat-engine retrieval: re-rank the query matches (sorted by id)
    with the user's mean-cosine scores (or popularity) and return them by descending score."""
    order = sorted(range(len(match_ids)), key=lambda i: match_ids[i])  # lib.py:75
    ids = [match_ids[i] for i in order]
    query_scores = pd.Series(data=[match_scores[i] for i in order], index=ids)
    query_movies = get_movies(tmdb_ids=ids)
    if user_id:
        user_scores = user_movie_scores(user_id, ids)
    else:
        user_scores = popularity_scores(query_movies)
    combined = reweight(query_scores, user_scores)
    recs = [Recommendation(movie=m, score=s) for m, s in zip(query_movies, combined)]
    return sorted(recs, key=lambda x: x.score, reverse=True)
