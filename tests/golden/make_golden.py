"""Generate the golden vectors that pin the oracle (and, through it, the GPU path).

Run in the build container only (it needs /root/reference; the GPU box never runs it):

    python tests/golden/make_golden.py

What it does
------------
1. Imports the reference's OWN hot-path module ``/root/reference/src/backend/app/lib.py``.
   Its import-time dependencies that are network/database clients absent from this image
   (``llama_index.llms`` message types, ``dotenv``, the CloudSQL connector, ``pg8000``) and the
   process-global resources module ``backend.app.constants`` (OpenAI/Chroma singletons) are
   replaced by inert stand-ins in ``sys.modules``. None of them is on the arithmetic path: the
   scoring runs the real scikit-learn ``cosine_similarity`` and the real pandas sort, exactly as
   ``lib.py:43-63`` calls them. The ratings table is the reference's own SQLAlchemy ``ratings``
   table (``database.py:83-90``) on an in-memory SQLite engine. ``get_movies`` (Postgres ARRAY
   columns, not creatable on SQLite) is replaced by a function returning ``Movie`` objects
   sorted by id -- the contract of ``lib.py:23-29``.
2. Calls ``lib.get_user_recs`` on a seeded synthetic collaborative catalog (the C1 shape,
   2269 x 32 float64) for 20 users, including the edge cases (no ratings, no liked movie,
   rated id absent from the catalog, a zero-norm catalog row, k larger than the candidates).
3. Calls ``lib.run_search`` with a stubbed chat engine returning fixed query matches, to pin
   the re-weighting arithmetic of ``lib.py:94-121``.
4. Computes ``sklearn.metrics.pairwise.cosine_similarity`` + ``pandas.Series.sort_values``
   top-K (the calls the reference makes) on seeded Gaussian data at small C2/C3-like shapes.

Inputs that are large are NOT stored: they are regenerated from the stored seeds by
``tests/golden/inputs.py`` (shared with the tests) and their SHA-256 is stored to detect drift.
"""
from __future__ import annotations

import json
import os
import sys
import types
from datetime import date, datetime

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"
sys.dont_write_bytecode = True  # the reference tree is read-only; never write bytecode there
sys.path.insert(0, HERE)

from inputs import (C1_SEED, COS_CASES, c1_catalog, c1_users, cos_case_inputs,  # noqa: E402
                    sha256_array)


def _install_stubs(catalog_df: pd.DataFrame, engine) -> None:
    """Inert stand-ins for the reference's I/O-client imports (not on the arithmetic path)."""
    llama = types.ModuleType("llama_index")
    llms = types.ModuleType("llama_index.llms")

    class MessageRole:
        USER = "user"
        ASSISTANT = "assistant"

    from pydantic import BaseModel

    class ChatMessage(BaseModel):  # the llama_index message type is a pydantic model too
        role: str = "user"
        content: str = ""

    llms.ChatMessage, llms.MessageRole = ChatMessage, MessageRole
    llama.llms = llms
    sys.modules["llama_index"], sys.modules["llama_index.llms"] = llama, llms

    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: None
    sys.modules["dotenv"] = dotenv
    google = types.ModuleType("google")
    cloud = types.ModuleType("google.cloud")
    sql = types.ModuleType("google.cloud.sql")
    conn = types.ModuleType("google.cloud.sql.connector")
    conn.Connector = object
    sys.modules.update({"google": google, "google.cloud": cloud, "google.cloud.sql": sql,
                        "google.cloud.sql.connector": conn})
    pg = types.ModuleType("pg8000")
    pg.Connection = object
    sys.modules["pg8000"] = pg

    consts = types.ModuleType("backend.app.constants")
    consts.engine = engine
    consts.openai_client = None
    consts.users_collab_collection = None
    consts.movies_collab_collection = None
    consts.movies_content_chat_engine = None
    consts.movies_collab_embeddings = catalog_df
    consts.LIKED_MOVIE_SCORE = 3.5
    consts.QUERY_SCORE_WEIGHT = 0.90
    consts.SIMILARITY_TOP_K = 10
    sys.modules["backend.app.constants"] = consts


def _movie(models, tmdb_id: str, popularity: float = 1.0):
    return models.Movie(tmdb_id=tmdb_id, tmdb_homepage="", title=f"t{tmdb_id}", language="en",
                        release_date=date(2000, 1, 1), runtime=90, director="d", actors=None,
                        genres=None, keywords=None, overview="", budget=0, revenue=0,
                        popularity=popularity, vote_average=0.0, vote_count=0)


def make_c1() -> dict:
    from sqlalchemy import create_engine, insert

    ids, cat = c1_catalog()
    catalog_df = pd.DataFrame(data=cat, index=ids)  # constants.py:55-56 (float64, str index)
    engine = create_engine("sqlite://")
    _install_stubs(catalog_df, engine)
    sys.path.insert(0, REF_SRC)
    from backend.app import database  # noqa: E402  (the reference's own tables)
    from backend.app import lib  # noqa: E402  (the reference's own hot path)
    from shared import models  # noqa: E402

    database.ratings.create(engine)
    users = c1_users(ids)
    with engine.begin() as cnx:
        for uid, rl in users.items():
            for tmdb_id, rating in rl:
                cnx.execute(insert(database.ratings).values(
                    user_id=uid, tmdb_id=tmdb_id, rating=rating, updated_at=datetime(2023, 1, 1)))

    # lib.py:23-29 contract: Movie rows for the ids, ORDER BY tmdb_id
    lib.get_movies = lambda tmdb_ids: [_movie(models, t) for t in sorted(tmdb_ids)]

    out = {"seed": C1_SEED, "catalog_sha256": sha256_array(cat), "users": {}}
    for uid, rl in users.items():
        rec = {"ratings": rl}
        for k in (10, 10000):
            try:
                recs = lib.get_user_recs(uid, k)
                rec[f"k{k}"] = [[r.movie.tmdb_id, float(r.score)] for r in recs]
            except ValueError as e:
                rec[f"k{k}"] = {"error": "ValueError", "message": str(e)}
        out["users"][uid] = rec

    # run_search re-weighting (lib.py:66-125) with a stubbed chat engine (LLM/Chroma absent)
    rng = np.random.default_rng(C1_SEED + 7)
    match_ids = sorted(rng.choice(ids, size=10, replace=False).tolist())
    match_scores = rng.uniform(0.70, 0.90, size=10).round(6).tolist()
    pops = rng.uniform(1.0, 100.0, size=10).round(3).tolist()

    class _Node:
        def __init__(self, node_id, score):
            self.node_id, self.score = node_id, score

    class _Resp:
        def __init__(self):
            self.response = "stub"
            self.source_nodes = [_Node(i, s) for i, s in zip(match_ids, match_scores)]

    class _Engine:
        def chat(self, message, chat_history):
            return _Resp()

    lib.movies_content_chat_engine = _Engine()
    popmap = dict(zip(match_ids, pops))
    lib.get_movies = lambda tmdb_ids: [_movie(models, t, popmap.get(t, 1.0)) for t in sorted(tmdb_ids)]
    msg = [sys.modules["llama_index.llms"].ChatMessage(content="q")]
    search = {"match_ids": match_ids, "match_scores": match_scores, "popularity": pops, "cases": {}}
    import contextlib
    import io
    for uid in [None] + [u for u in users if users[u]][:4]:
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                resp = lib.run_search(msg, user_id=uid)
            search["cases"][str(uid)] = [[r.movie.tmdb_id, float(r.score)] for r in resp.recommendations]
        except (ValueError, KeyError) as e:
            search["cases"][str(uid)] = {"error": type(e).__name__, "message": str(e)}
    out["search"] = search
    return out


def make_cos_cases() -> dict:
    from sklearn.metrics.pairwise import cosine_similarity

    out = {}
    arrays = {}
    for name, case in COS_CASES.items():
        q, c, excl = cos_case_inputs(case)
        sims = cosine_similarity(q, c)  # float64 (both inputs float64)
        K = case["k"]
        rows = np.full((q.shape[0], K), -1, dtype=np.int64)
        scores = np.full((q.shape[0], K), np.nan)
        for b in range(q.shape[0]):
            s = pd.Series(sims[b])
            if excl is not None:
                s = s.loc[s.index.difference(pd.Index(excl[b]))]
            top = s.sort_values(ascending=False)[:K]  # lib.py:55
            rows[b, :len(top)] = top.index.values
            scores[b, :len(top)] = top.values
        arrays[f"{name}_rows"] = rows.astype(np.int32)
        arrays[f"{name}_scores"] = scores
        out[name] = dict(case, q_sha256=sha256_array(q), c_sha256=sha256_array(c))
    np.savez_compressed(os.path.join(HERE, "cos_topk_small.npz"), **arrays)
    return out


def main() -> None:
    c1 = make_c1()
    with open(os.path.join(HERE, "c1_collab.json"), "w") as f:
        json.dump(c1, f, indent=1)
    cases = make_cos_cases()
    with open(os.path.join(HERE, "cos_topk_small.json"), "w") as f:
        json.dump(cases, f, indent=1)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
