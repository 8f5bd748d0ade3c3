"""Throughput and latency of the recommend route's request path under the
reference's concurrency: FastAPI runs the sync handler of
/root/reference/src/backend/app/api/users.py:150-155 on up to 40 anyio worker threads, one user
per call (lib.py:32-63). Here 40 request threads drive

  * route:   lib.get_user_recs_batched (the same SQL on a file-backed SQLite ratings table, the
             pandas filtering, the scoring coalesced by one batcher.RecBatcher, the hydration);
  * scoring: RecBatcher.submit(liked, rated, k) alone (the GPU path without SQL / hydration);

for --seconds each, and report requests/s, p50 / p99 latency and the batch-size histogram, beside
  * unbatched: lib.get_user_recs one call at a time (B = 1 through the C ABI);
  * reference CPU: the float64 oracle restatement of lib.py:51-55 per call (cosine_similarity
    re-normalising the catalog, mean, exclusion, sort; oracle.restatement.liked_topk) on a bounded
    sample -- the reference's own per-request arithmetic on this host.
Shapes: C1 = the reference's movie table shape (2269 x 32 float64); C3 = 1M x 1536 float32 with
users of --liked liked rows. Synthetic data (seeded Gaussian catalog, random ratings).

    python tools/route_bench.py --shape C1 [--threads 40 --seconds 10 --users 2000 --k 10]
"""
import argparse
import concurrent.futures as cf
import datetime
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import lib, tables  # noqa: E402
from robot_ebert_amd.batcher import RecBatcher  # noqa: E402
from robot_ebert_amd.models import Movie  # noqa: E402

SHAPES = {"C1": dict(n=2269, d=32, dtype=torch.float64),
          "C3": dict(n=1_000_000, d=1536, dtype=torch.float32)}


def setup(shape, users, liked, rated, seed=0):
    import tempfile
    from sqlalchemy import create_engine, insert
    cfg = SHAPES[shape]
    n, d = cfg["n"], cfg["d"]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(seed)
    emb = torch.randn((n, d), generator=g, device=dev, dtype=torch.float32).to(cfg["dtype"])
    ids = [str(100000 + i) for i in range(n)]
    cat = ebt.Catalog(emb, ids=ids)
    rng = np.random.default_rng(seed + 1)
    # a file-backed SQLite database: one connection per request thread (the reference's
    # Postgres pool serves its 40 worker threads concurrently as well)
    path = os.path.join(tempfile.mkdtemp(), "ratings.db")
    engine = create_engine(f"sqlite:///{path}", connect_args={"check_same_thread": False},
                           pool_size=64, max_overflow=0)
    tables.ratings.create(engine)
    user_rows = {}
    rows = []
    for u in range(users):
        pick = rng.choice(n, liked + rated, replace=False)
        uid = f"u{u}"
        user_rows[uid] = (sorted(pick[:liked].tolist()), sorted(pick.tolist()))
        for j, r in enumerate(pick):
            rt = float(rng.uniform(4.0, 5.0)) if j < liked else float(rng.uniform(0.5, 3.0))
            rows.append(dict(user_id=uid, tmdb_id=ids[r], rating=rt))
    with engine.begin() as cnx:
        cnx.execute(insert(tables.ratings), rows)

    def movies(tmdb_ids):
        return [Movie(tmdb_id=t, tmdb_homepage="", title=t, language="en",
                      release_date=datetime.date(2000, 1, 1), runtime=90, director="d",
                      actors=None, genres=None, keywords=None, overview="", budget=0, revenue=0,
                      popularity=1.0, vote_average=0.0, vote_count=0) for t in sorted(tmdb_ids)]
    lib.configure(engine=engine, catalog=cat, get_movies=movies)
    return cat, emb, user_rows


def drive(fn, uids, threads, seconds):
    """`threads` threads calling fn(uid) in a loop for `seconds`; (requests, latencies s)."""
    lat = [[] for _ in range(threads)]
    stop = time.monotonic() + seconds
    start = threading.Barrier(threads)

    def worker(t):
        rng = np.random.default_rng(t)
        start.wait()
        while time.monotonic() < stop:
            uid = uids[int(rng.integers(len(uids)))]
            t0 = time.perf_counter()
            fn(uid)
            lat[t].append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(worker, range(threads)))
    el = time.perf_counter() - t0
    flat = np.concatenate([np.asarray(x) for x in lat])
    return len(flat), el, flat


def summary(n, el, lat):
    return {"requests": int(n), "seconds": round(el, 2), "req_per_s": round(n / el, 1),
            "p50_ms": round(float(np.percentile(lat, 50)) * 1e3, 3),
            "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="C1", choices=sorted(SHAPES))
    ap.add_argument("--threads", type=int, default=40)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--users", type=int, default=2000)
    ap.add_argument("--liked", type=int, default=20)
    ap.add_argument("--rated", type=int, default=30)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--max-wait-ms", type=float, default=1.0)
    ap.add_argument("--cpu-calls", type=int, default=0, help="reference CPU sample (0: auto)")
    a = ap.parse_args()
    ebt.load()
    cat, emb, user_rows = setup(a.shape, a.users, a.liked, a.rated)
    uids = list(user_rows)
    k = a.k
    out = {"shape": a.shape, "n": cat.n, "d": cat.d, "dtype": str(emb.dtype), "users": a.users,
           "liked_per_user": a.liked, "rated_per_user": a.liked + a.rated, "k": k,
           "threads": a.threads, "max_wait_ms": a.max_wait_ms,
           "data": "synthetic (seeded Gaussian catalog, random ratings in a file-backed SQLite table)"}
    # warm
    for u in uids[:3]:
        lib.get_user_recs(u, k)
    torch.cuda.synchronize()
    # unbatched: one call at a time
    t0 = time.perf_counter()
    m = 0
    lats = []
    while time.perf_counter() - t0 < min(5.0, a.seconds) or m < 5:
        t1 = time.perf_counter()
        lib.get_user_recs(uids[m % len(uids)], k)
        lats.append(time.perf_counter() - t1)
        m += 1
    out["unbatched_route"] = summary(m, time.perf_counter() - t0, np.asarray(lats))

    for mode in ("scoring", "route"):
        b = RecBatcher(cat, max_batch=4096, max_wait_ms=a.max_wait_ms)
        if mode == "route":
            def fn(uid, b=b):
                lib.get_user_recs_batched(b, uid, k)
        else:
            def fn(uid, b=b):
                liked, rated = user_rows[uid]
                b.submit(liked, rated, k).result()
        fn(uids[0])
        n, el, lat = drive(fn, uids, a.threads, a.seconds)
        b.close()
        st = b.stats()
        out[f"batched_{mode}"] = dict(summary(n, el, lat), mean_batch=round(st["mean_batch"], 2),
                                      batch_size_hist_pow2=st["size_hist_pow2"])
        print(f"{mode}: {out[f'batched_{mode}']}", file=sys.stderr, flush=True)

    # correctness of a few batched answers against the unbatched path (same arithmetic)
    b = RecBatcher(cat, max_batch=64, max_wait_ms=5.0)
    with cf.ThreadPoolExecutor(16) as ex:
        got = list(ex.map(lambda u: lib.get_user_recs_batched(b, u, k), uids[:32]))
    b.close()
    same = all([(g.movie.tmdb_id, g.score) for g in x] ==
               [(g.movie.tmdb_id, g.score) for g in lib.get_user_recs(u, k)]
               for x, u in zip(got, uids[:32]))
    out["batched_equals_unbatched_32_users"] = bool(same)

    # the reference's per-request CPU arithmetic (float64 oracle restatement of lib.py:51-55)
    sys.path.insert(0, ROOT)
    from oracle import restatement as R
    c64 = emb.double().cpu().numpy()
    calls = a.cpu_calls or (200 if cat.n < 10000 else 3)
    t0 = time.perf_counter()
    for i in range(calls):
        liked, rated = user_rows[uids[i % len(uids)]]
        R.liked_topk(c64, [liked], k, [rated])
    el = time.perf_counter() - t0
    out["reference_cpu_per_call"] = {"calls": calls, "ms_per_call": round(el / calls * 1e3, 3),
                                     "req_per_s_one_thread": round(calls / el, 2),
                                     "what": "oracle.restatement.liked_topk (float64, "
                                             "cosine_similarity of the liked rows vs the "
                                             "catalog, mean, exclusion, sort), one call at a "
                                             "time on this host"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
