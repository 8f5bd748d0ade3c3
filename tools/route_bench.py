"""Throughput and latency of the recommend route's request path under the
reference's concurrency: FastAPI runs the sync handler of
/root/reference/src/backend/app/api/users.py:150-155 on up to 40 anyio worker threads, one user
per call (lib.py:32-63). Here request threads drive

  * unbatched: lib.get_user_recs one call at a time, and from --threads threads (B = 1 through the
               C ABI per request);
  * scoring:   RecBatcher.submit(liked, rated, k) alone (the GPU path without SQL / hydration);
  * route:     lib.get_user_recs_batched in ONE process (the same SQL on a file-backed SQLite
               ratings table, the filtering, the scoring coalesced by one batcher.RecBatcher,
               the hydration), with the CPU time of every thread of the process over the run
               (psutil: request threads, the batcher's dispatcher and completion threads) --
               where the interpreter time goes;
  * multiproc: --workers P server processes of --threads / P request threads each (the same
               route code over a CatalogIndex, no GPU), scoring through ONE GPU-owning process
               (serving.ScoreServer over a RecBatcher, Unix socket) -- the deployment shape;

for --seconds each, and report requests/s, p50 / p99 latency and the batch-size histogram, beside
the reference's per-request float64 arithmetic (the oracle restatement of lib.py:51-55) on a
bounded sample. Shapes: C1 = the reference's movie table shape (2269 x 32 float64); C3 = 1M x
1536 float32 with users of --liked liked rows. Synthetic data (seeded Gaussian catalog, random
ratings). The worker processes are started before this process touches the GPU.

    python tools/route_bench.py --shape C3 [--threads 40 --seconds 10 --workers 4 --k 10]
"""
import argparse
import concurrent.futures as cf
import datetime
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"C1": dict(n=2269, d=32, dtype="float64"),
          "C3": dict(n=1_000_000, d=1536, dtype="float32")}


def catalog_ids(n):
    return [str(100000 + i) for i in range(n)]


def setup_db(shape, users, liked, rated, path, seed=0):
    """The ratings table (file-backed SQLite, no GPU): user -> (liked rows, rated rows)."""
    from sqlalchemy import create_engine, insert
    from robot_ebert_amd import tables
    n = SHAPES[shape]["n"]
    ids = catalog_ids(n)
    rng = np.random.default_rng(seed + 1)
    engine = create_engine(f"sqlite:///{path}")
    tables.ratings.create(engine)
    user_rows, rows = {}, []
    for u in range(users):
        pick = rng.choice(n, liked + rated, replace=False)
        uid = f"u{u}"
        user_rows[uid] = (sorted(pick[:liked].tolist()), sorted(pick.tolist()))
        for j, r in enumerate(pick):
            rt = float(rng.uniform(4.0, 5.0)) if j < liked else float(rng.uniform(0.5, 3.0))
            rows.append(dict(user_id=uid, tmdb_id=ids[r], rating=rt))
    with engine.begin() as cnx:
        cnx.execute(insert(tables.ratings), rows)
    engine.dispose()
    return user_rows


def open_engine(path):
    # one connection per request thread (the reference's Postgres pool serves its 40 worker
    # threads concurrently as well)
    from sqlalchemy import create_engine
    return create_engine(f"sqlite:///{path}", connect_args={"check_same_thread": False},
                         pool_size=64, max_overflow=0)


def movies(tmdb_ids):
    from robot_ebert_amd.models import Movie
    return [Movie(tmdb_id=t, tmdb_homepage="", title=t, language="en",
                  release_date=datetime.date(2000, 1, 1), runtime=90, director="d",
                  actors=None, genres=None, keywords=None, overview="", budget=0, revenue=0,
                  popularity=1.0, vote_average=0.0, vote_count=0) for t in sorted(tmdb_ids)]


def drive(fn, uids, threads, seconds, cpu=None):
    """`threads` threads calling fn(uid) in a loop for `seconds`; (requests, elapsed s, latencies).
    cpu (a list): gets the request threads' CPU seconds (time.thread_time of each) appended."""
    lat = [[] for _ in range(threads)]
    tcpu = [0.0] * threads
    stop = time.monotonic() + seconds
    start = threading.Barrier(threads)

    def worker(t):
        rng = np.random.default_rng(t + 1000 * os.getpid())
        start.wait()
        c0 = time.thread_time()
        while time.monotonic() < stop:
            uid = uids[int(rng.integers(len(uids)))]
            t0 = time.perf_counter()
            fn(uid)
            lat[t].append(time.perf_counter() - t0)
        tcpu[t] = time.thread_time() - c0
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(worker, range(threads)))
    el = time.perf_counter() - t0
    if cpu is not None:
        cpu.append(sum(tcpu))
    flat = np.concatenate([np.asarray(x) for x in lat])
    return len(flat), el, flat


def summary(n, el, lat):
    return {"requests": int(n), "seconds": round(el, 2), "req_per_s": round(n / el, 1),
            "p50_ms": round(float(np.percentile(lat, 50)) * 1e3, 3),
            "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 3)}


def thread_cpu():
    """{native thread id: user + system CPU seconds} of this process (psutil)."""
    import psutil
    return {t.id: t.user_time + t.system_time for t in psutil.Process().threads()}


def cpu_by_role(before, after, names):
    """CPU seconds of the named long-lived threads (the batcher's dispatcher / completion
    threads) over a run (the request threads are measured by drive itself)."""
    out = {}
    for tid, role in names.items():
        out[role] = out.get(role, 0.0) + after.get(tid, 0.0) - before.get(tid, 0.0)
    return {k: round(v, 3) for k, v in out.items()}


# ------------------------------------------------------------------ worker process ----------
def worker_main(a):
    """One route server process: the route's host work over a CatalogIndex, scoring through
    the GPU-owning process's ScoreServer. Prints one JSON line; latencies to --lat-out."""
    from robot_ebert_amd import lib
    from robot_ebert_amd.serving import CatalogIndex, ScoreClient
    cfg = SHAPES[a.shape]
    ix = CatalogIndex(catalog_ids(cfg["n"]), cfg["d"])
    ix.index_pos   # built before the clock starts
    lib.configure(engine=open_engine(a.db), catalog=ix, get_movies=movies)
    uids = [f"u{u}" for u in range(a.users)]
    t_end = time.monotonic() + 600
    while not os.path.exists(a.address) and time.monotonic() < t_end:
        time.sleep(0.02)
    client = ScoreClient(a.address)
    for u in uids[:3]:
        lib.get_user_recs_batched(client, u, a.k)
    with open(a.address + f".ready{a.worker}", "w"):
        pass
    while not os.path.exists(a.address + ".go") and time.monotonic() < t_end:
        time.sleep(0.005)
    n, el, lat = drive(lambda uid: lib.get_user_recs_batched(client, uid, a.k), uids,
                       a.threads, a.seconds)
    np.save(a.lat_out, lat)
    client.close()
    print(json.dumps(dict(summary(n, el, lat), worker=a.worker)), flush=True)


def multiproc(a, db, procs, cat, uids, k):
    """The GPU side of the multiproc mode: serve the already started worker processes."""
    from robot_ebert_amd.batcher import RecBatcher
    from robot_ebert_amd.serving import ScoreServer
    b = RecBatcher(cat, max_batch=4096, max_wait_ms=a.max_wait_ms)
    srv = ScoreServer(b, address=a.sock)
    t_end = time.monotonic() + 300
    while time.monotonic() < t_end and not all(
            os.path.exists(a.sock + f".ready{w}") for w in range(a.workers)):
        if any(p.poll() not in (None, 0) for p in procs):
            raise SystemExit("a worker process failed during start-up")
        time.sleep(0.05)
    st0 = b.stats()
    with open(a.sock + ".go", "w"):
        pass
    res = []
    for p in procs:
        out, _ = p.communicate(timeout=a.seconds + 300)
        if p.returncode != 0:
            raise SystemExit(f"worker exited with {p.returncode}")
        res.append(json.loads(out.strip().splitlines()[-1]))
    srv.close()
    b.close()
    st = b.stats()
    lat = np.concatenate([np.load(os.path.join(os.path.dirname(a.sock), f"lat{w}.npy"))
                          for w in range(a.workers)])
    n = sum(r["requests"] for r in res)
    el = max(r["seconds"] for r in res)
    nb = st["batches"] - st0["batches"]
    return dict(summary(n, el, lat), workers=a.workers,
                threads_per_worker=a.threads // a.workers,
                mean_batch=round((st["requests"] - st0["requests"]) / max(nb, 1), 2),
                per_worker_req_per_s=[r["req_per_s"] for r in res],
                batch_size_hist_pow2=st["size_hist_pow2"])


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
    ap.add_argument("--workers", type=int, default=0,
                    help="multiproc mode: route server processes (threads split among them)")
    ap.add_argument("--modes", default="unbatched,scoring,route,multiproc")
    ap.add_argument("--cpu-calls", type=int, default=0, help="reference CPU sample (0: auto)")
    ap.add_argument("--worker", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--db", help=argparse.SUPPRESS)
    ap.add_argument("--address", help=argparse.SUPPRESS)
    ap.add_argument("--lat-out", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.worker >= 0:
        return worker_main(a)
    modes = a.modes.split(",")
    tmp = tempfile.mkdtemp(prefix="route_bench_")
    db = os.path.join(tmp, "ratings.db")
    user_rows = setup_db(a.shape, a.users, a.liked, a.rated, db)
    uids = list(user_rows)
    k = a.k
    procs = []
    if a.workers > 0 and "multiproc" in modes:
        # started before this process touches the GPU (they never do)
        a.sock = os.path.join(tmp, "score.sock")
        per = max(1, a.threads // a.workers)
        for w in range(a.workers):
            cmd = [sys.executable, os.path.abspath(__file__), "--worker", str(w), "--db", db,
                   "--address", a.sock, "--shape", a.shape, "--threads", str(per),
                   "--seconds", str(a.seconds), "--users", str(a.users), "--k", str(k),
                   "--lat-out", os.path.join(tmp, f"lat{w}.npy")]
            procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True))

    import torch
    import robot_ebert_amd as ebt
    from robot_ebert_amd import lib
    from robot_ebert_amd.batcher import RecBatcher
    ebt.load()
    cfg = SHAPES[a.shape]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    emb = torch.randn((cfg["n"], cfg["d"]), generator=g, device=dev,
                      dtype=torch.float32).to(getattr(torch, cfg["dtype"]))
    cat = ebt.Catalog(emb, ids=catalog_ids(cfg["n"]))
    cat.index_pos
    lib.configure(engine=open_engine(db), catalog=cat, get_movies=movies)
    out = {"shape": a.shape, "n": cat.n, "d": cat.d, "dtype": str(emb.dtype), "users": a.users,
           "liked_per_user": a.liked, "rated_per_user": a.liked + a.rated, "k": k,
           "threads": a.threads, "max_wait_ms": a.max_wait_ms,
           "host_cpus": os.cpu_count(),
           "data": "synthetic (seeded Gaussian catalog, random ratings in a file-backed SQLite table)"}
    for u in uids[:3]:
        lib.get_user_recs(u, k)
    torch.cuda.synchronize()
    try:
        if "multiproc" in modes and procs:
            out["multiproc_route"] = multiproc(a, db, procs, cat, uids, k)
            print(f"multiproc: {out['multiproc_route']}", file=sys.stderr, flush=True)
        if "unbatched" in modes:
            t0 = time.perf_counter()
            m, lats = 0, []
            while time.perf_counter() - t0 < min(5.0, a.seconds) or m < 5:
                t1 = time.perf_counter()
                lib.get_user_recs(uids[m % len(uids)], k)
                lats.append(time.perf_counter() - t1)
                m += 1
            out["unbatched_route"] = summary(m, time.perf_counter() - t0, np.asarray(lats))
            req_cpu = []
            n, el, lat = drive(lambda uid: lib.get_user_recs(uid, k), uids, a.threads, a.seconds,
                               cpu=req_cpu)
            out[f"unbatched_route_{a.threads}_threads"] = dict(
                summary(n, el, lat), cpu_ms_per_request=round(1e3 * req_cpu[0] / max(n, 1), 3))
            print(f"unbatched: {out[f'unbatched_route_{a.threads}_threads']}", file=sys.stderr,
                  flush=True)
        for mode in ("scoring", "route"):
            if mode not in modes:
                continue
            b = RecBatcher(cat, max_batch=4096, max_wait_ms=a.max_wait_ms)
            if mode == "route":
                def fn(uid, b=b):
                    lib.get_user_recs_batched(b, uid, k)
            else:
                def fn(uid, b=b):
                    liked, rated = user_rows[uid]
                    b.submit(liked, rated, k).result()
            fn(uids[0])
            names = {b._thread.native_id: "batcher dispatcher"}
            if b._completer is not None:
                names[b._completer.native_id] = "batcher completion"
            c0 = thread_cpu()
            req_cpu = []
            n, el, lat = drive(fn, uids, a.threads, a.seconds, cpu=req_cpu)
            cpu = cpu_by_role(c0, thread_cpu(), names)
            cpu["request threads"] = round(req_cpu[0], 3)
            b.close()
            st = b.stats()
            out[f"batched_{mode}"] = dict(
                summary(n, el, lat), mean_batch=round(st["mean_batch"], 2),
                batch_size_hist_pow2=st["size_hist_pow2"], cpu_s_by_thread_role=cpu,
                cpu_ms_per_request={r: round(1e3 * v / max(n, 1), 3) for r, v in cpu.items()})
            print(f"{mode}: {out[f'batched_{mode}']}", file=sys.stderr, flush=True)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()

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
