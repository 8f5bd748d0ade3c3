"""CPU: multi-process serving of the recommend route (robot_ebert_amd/serving.py).

The GPU-owning side (``ScoreServer`` over a ``RecBatcher``) runs here with the float64 oracle
injected as the batcher's scoring function (test infrastructure standing in for the GPU
``score_topk``); clients connect over the Unix socket from threads of this process and from a
separate Python process (the route's server processes). Checked: answers equal the oracle for
every request, requests of several clients share batches, per-request errors keep their type,
a malformed frame only ends its own connection, and closing the server fails the pending
callers instead of hanging them.
"""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from oracle import restatement as R
from robot_ebert_amd.batcher import RecBatcher
from robot_ebert_amd.serving import (CatalogIndex, ScoreClient, ScoreServer, decode_request,
                                     decode_response, encode_request, encode_response)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Cat:
    def __init__(self, x):
        self.x, self.d = x, x.shape[1]


def _oracle_score(calls):
    def score(cat, k, liked, exclude):
        calls.append(len(liked))
        qs = np.stack([R.mean_cosine_query(cat.x[l]) for l in liked])
        return R.cosine_topk(qs, cat.x, k, exclude)
    return score


def _direct(x, liked, excl, k):
    s, r = R.cosine_topk(R.mean_cosine_query(x[liked])[None, :], x, k, [excl])
    keep = r[0] >= 0
    return s[0][keep], r[0][keep]


def test_wire_roundtrip():
    f = encode_request(7, [3, 1, 2], [9], 5)
    rid, k, lk, rt = decode_request(f)
    assert (rid, k, lk.tolist(), rt.tolist()) == (7, 5, [3, 1, 2], [9])
    rid, (s, r) = decode_response(encode_response(9, np.array([0.5, 0.25]), np.array([4, 2])))
    assert rid == 9 and s.tolist() == [0.5, 0.25] and r.tolist() == [4, 2]
    for e in (ValueError("Found array with 0 sample(s)"), KeyError("tmdb_id"), MemoryError("x")):
        rid, got = decode_response(encode_response(3, exc=e))
        assert rid == 3 and isinstance(got, ValueError if isinstance(e, ValueError) else
                                       KeyError if isinstance(e, KeyError) else RuntimeError)
    with pytest.raises(ValueError):
        decode_request(f[:-3])


def test_catalog_index_matches_catalog_semantics():
    ids = ["862", "10", "2"]
    ix = CatalogIndex(ids, d=4, row_offset=100)
    assert ix.rows_of(["2", "862"]) == [102, 100] and ix.id_of(101) == "10"
    assert ix.contains(["10", "11"]) == [True, False]
    with pytest.raises(KeyError):
        ix.rows_of(["11"])


def test_threads_of_several_clients_share_batches():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((600, 16))
    calls = []
    b = RecBatcher(_Cat(x), max_batch=64, max_wait_ms=20.0, score_fn=_oracle_score(calls))
    srv = ScoreServer(b)
    clients = [ScoreClient(srv.address) for _ in range(3)]
    reqs = [(sorted(rng.choice(600, 3, replace=False).tolist()),
             sorted(rng.choice(600, 10, replace=False).tolist()), int(k))
            for k in rng.integers(1, 30, 60)]
    out = [None] * len(reqs)

    def worker(i):
        c = clients[i % 3]
        out[i] = c.score(*reqs[i])
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(len(reqs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    for (liked, excl, k), (s, r) in zip(reqs, out):
        ws, wr = _direct(x, liked, excl, k)
        np.testing.assert_array_equal(r, wr)
        np.testing.assert_allclose(s, ws, rtol=0, atol=1e-15)
    assert sum(calls) == len(reqs) and max(calls) > 1   # coalesced across clients
    # per-request errors keep their type; the connection stays usable
    with pytest.raises(ValueError, match="0 sample"):
        clients[0].score([], [1], 3)
    assert len(clients[0].score([5], [], 4)[1]) == 4
    for c in clients:
        c.close()
    srv.close()
    b.close()


def test_malformed_frame_ends_only_its_connection():
    from multiprocessing.connection import Client
    from robot_ebert_amd.serving import AUTHKEY
    x = np.random.default_rng(1).standard_normal((100, 8))
    b = RecBatcher(_Cat(x), max_batch=8, max_wait_ms=1.0, score_fn=_oracle_score([]))
    srv = ScoreServer(b)
    bad = Client(srv.address, family="AF_UNIX", authkey=AUTHKEY)
    bad.send_bytes(b"\x00" * 5)
    rid, err = decode_response(bad.recv_bytes())
    assert isinstance(err, RuntimeError) or isinstance(err, Exception)
    with pytest.raises(EOFError):
        bad.recv_bytes()
    good = ScoreClient(srv.address)
    assert len(good.score([1, 2], [3], 5)[1]) == 5
    good.close()
    srv.close()
    b.close()


def test_client_that_stops_reading_does_not_block_others():
    """A connection whose client never reads its answers (its socket buffer full) blocks only
    its own writer: the batcher's completion thread and the other clients go on."""
    from multiprocessing.connection import Client
    from robot_ebert_amd.serving import AUTHKEY
    x = np.random.default_rng(5).standard_normal((6000, 8))
    b = RecBatcher(_Cat(x), max_batch=8, max_wait_ms=1.0, score_fn=_oracle_score([]))
    srv = ScoreServer(b)
    stuck = Client(srv.address, family="AF_UNIX", authkey=AUTHKEY)
    for i in range(40):   # 40 answers of 5000 rows (80 KB each): far more than a socket buffer
        stuck.send_bytes(encode_request(i + 1, [1, 2], [], 5000))
    good = ScoreClient(srv.address, timeout=30.0)
    for i in range(5):
        assert len(good.score([3 + i], [], 7)[1]) == 7
    good.close()
    srv.close()
    stuck.close()
    b.close()


def test_server_close_fails_pending_callers():
    x = np.random.default_rng(2).standard_normal((100, 8))
    gate = threading.Event()

    def slow(cat, k, liked, exclude):
        gate.wait(10)
        return _oracle_score([])(cat, k, liked, exclude)
    b = RecBatcher(_Cat(x), max_batch=8, max_wait_ms=1.0, score_fn=slow)
    srv = ScoreServer(b)
    c = ScoreClient(srv.address, timeout=10.0)
    fut = c.submit([1], [], 3)
    srv.close()
    with pytest.raises(RuntimeError, match="closed"):
        fut.result(timeout=10)
    gate.set()
    b.close()
    c.close()


_CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
from robot_ebert_amd.serving import ScoreClient
import concurrent.futures as cf
reqs = json.loads(sys.argv[2])
c = ScoreClient(sys.argv[1])
with cf.ThreadPoolExecutor(8) as ex:
    res = list(ex.map(lambda q: c.score(*q), reqs))
print(json.dumps([[s.tolist(), r.tolist()] for s, r in res]))
c.close()
"""


def test_client_in_another_process():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((500, 12))
    b = RecBatcher(_Cat(x), max_batch=32, max_wait_ms=5.0, score_fn=_oracle_score([]))
    srv = ScoreServer(b)
    # three liked rows (two would tie exactly with each other, cos(q, x_a) = cos(q, x_b), and
    # the oracle's batched / single forms break such a tie by round-off differently)
    reqs = [(sorted(rng.choice(500, 3, replace=False).tolist()),
             sorted(rng.choice(500, 6, replace=False).tolist()), 7) for _ in range(24)]
    p = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT), srv.address,
                        json.dumps(reqs)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    got = json.loads(p.stdout)
    for (liked, excl, k), (s, r) in zip(reqs, got):
        ws, wr = _direct(x, liked, excl, k)
        assert r == wr.tolist()
        np.testing.assert_allclose(s, ws, rtol=0, atol=1e-15)
    srv.close()
    b.close()


def test_route_through_the_score_server(monkeypatch, tmp_path):
    """lib.get_user_recs_batched in a route server process's shape: the same SQL (file-backed
    SQLite), filtering and hydration over a CatalogIndex (no embeddings), scoring through a
    ScoreClient -- the same Recommendations as the in-process batcher, the sklearn error text for
    a user without liked movies, [] for a user without ratings."""
    import datetime
    import concurrent.futures as cf
    from sqlalchemy import create_engine, insert
    from robot_ebert_amd import lib, tables
    from robot_ebert_amd.models import Movie

    rng = np.random.default_rng(4)
    n, d = 400, 16
    x = rng.standard_normal((n, d))
    ids = [str(1000 + i) for i in range(n)]
    eng = create_engine(f"sqlite:///{tmp_path / 'r.db'}",
                        connect_args={"check_same_thread": False})
    tables.ratings.create(eng)
    rows = []
    for u in range(12):
        pick = rng.choice(n, 8, replace=False)
        for j, r in enumerate(pick):
            rows.append(dict(user_id=f"u{u}", tmdb_id=ids[r],
                             rating=4.5 if j < 3 else 2.0))
    rows += [dict(user_id="nolike", tmdb_id=ids[5], rating=1.0)]
    with eng.begin() as cnx:
        cnx.execute(insert(tables.ratings), rows)

    def movies(tmdb_ids):
        return [Movie(tmdb_id=t, tmdb_homepage="", title=t, language="en",
                      release_date=datetime.date(2000, 1, 1), runtime=90, director="d",
                      actors=None, genres=None, keywords=None, overview="", budget=0, revenue=0,
                      popularity=1.0, vote_average=0.0, vote_count=0) for t in sorted(tmdb_ids)]
    for name in ("engine", "movies_collab_catalog", "_get_movies_override"):
        monkeypatch.setattr(lib, name, getattr(lib, name))
    lib.configure(engine=eng, catalog=CatalogIndex(ids, d), get_movies=movies)
    direct = RecBatcher(_Cat(x), max_batch=16, max_wait_ms=2.0, score_fn=_oracle_score([]))
    b = RecBatcher(_Cat(x), max_batch=16, max_wait_ms=2.0, score_fn=_oracle_score([]))
    srv = ScoreServer(b)
    client = ScoreClient(srv.address)
    uids = [f"u{u}" for u in range(12)]
    with cf.ThreadPoolExecutor(6) as ex:
        got = list(ex.map(lambda u: lib.get_user_recs_batched(client, u, 5), uids))
    want = [lib.get_user_recs_batched(direct, u, 5) for u in uids]
    for g, w in zip(got, want):   # (the oracle's batched BLAS rounds by batch composition)
        assert [r.movie.tmdb_id for r in g] == [r.movie.tmdb_id for r in w]
        np.testing.assert_allclose([r.score for r in g], [r.score for r in w], rtol=0, atol=1e-15)
        assert len(g) == 5
    with pytest.raises(ValueError, match="0 sample"):
        lib.get_user_recs_batched(client, "nolike", 5)
    assert lib.get_user_recs_batched(client, "nobody", 5) == []
    client.close()
    srv.close()
    b.close()
    direct.close()


def test_cancelled_future_does_not_stop_the_client():
    """A caller that cancels its Future before the answer arrives: the client's reader drops
    that answer and goes on resolving the others (a set_result on a cancelled Future would raise
    in the reader and leave every later request hanging)."""
    x = np.random.default_rng(6).standard_normal((200, 8))
    gate = threading.Event()

    def slow(cat, k, liked, exclude):
        gate.wait(10)
        return _oracle_score([])(cat, k, liked, exclude)
    b = RecBatcher(_Cat(x), max_batch=8, max_wait_ms=1.0, score_fn=slow)
    srv = ScoreServer(b)
    c = ScoreClient(srv.address, timeout=20.0)
    f1 = c.submit([1], [], 3)
    assert f1.cancel()
    gate.set()
    for i in range(4):
        assert len(c.score([2 + i], [], 4)[1]) == 4
    c.close()
    srv.close()
    b.close()


def test_garbled_server_frame_fails_pending_callers(tmp_path):
    """A frame from the server that does not decode ends the client's connection: its pending
    and later callers get a RuntimeError instead of waiting forever (the reader thread must not
    die with callers registered)."""
    from multiprocessing.connection import Listener
    from robot_ebert_amd.serving import AUTHKEY
    addr = str(tmp_path / "fake.sock")
    lst = Listener(addr, family="AF_UNIX", authkey=AUTHKEY)
    got = {}

    def fake_server():
        conn = lst.accept()
        got["req"] = conn.recv_bytes()
        conn.send_bytes(b"\x01\x02")        # shorter than a response header
        try:
            conn.recv_bytes()               # until the client shuts the connection down
        except (OSError, EOFError):
            pass
        conn.close()
    t = threading.Thread(target=fake_server)
    t.start()
    c = ScoreClient(addr, timeout=10.0)
    f = c.submit([1], [], 3)
    with pytest.raises(RuntimeError, match="malformed|closed"):
        f.result(timeout=10.0)
    with pytest.raises(RuntimeError):
        c.score([2], [], 3)
    c.close()
    t.join(10)
    lst.close()
    assert decode_request(got["req"])[0] == 1


def test_bad_request_fails_only_itself():
    """a request is checked before it can share a batch. One client's liked row past
    the catalog fails only that request (the library would reject the whole batch: a liked row
    out of range is EBT_EINVAL for the call), while another client's request coalesced in the
    same window is answered; a huge k is clamped to the catalog (same answer), rated rows outside
    the catalog are ignored (lib.py:48's index.difference ignores unknown ids)."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((300, 8))

    class Cat(_Cat):
        n, n_global, row_offset = 300, 300, 0

    calls = []
    inner = _oracle_score(calls)

    def strict(cat, k, liked, exclude):     # the library's own argument checks
        if any(r < 0 or r >= cat.n for l in liked for r in l) or k > 100_000:
            raise ValueError("the whole batch was rejected")
        return inner(cat, k, liked, exclude)
    b = RecBatcher(Cat(x), max_batch=64, max_wait_ms=200.0, score_fn=strict)
    srv = ScoreServer(b)
    ca, cb = ScoreClient(srv.address), ScoreClient(srv.address)
    res = {}

    def run(name, c, args):
        try:
            res[name] = c.score(*args)
        except Exception as e:  # noqa: BLE001
            res[name] = e
    good = ([3, 7], [1, 2, 5000], (1 << 31) - 1)     # the wire's largest k
    ts = [threading.Thread(target=run, args=("bad", ca, ([3, 300], [], 5))),
          threading.Thread(target=run, args=("good", cb, good)),
          threading.Thread(target=run, args=("neg", ca, ([-1], [], 5)))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert isinstance(res["bad"], ValueError) and "not in the catalog" in str(res["bad"])
    assert isinstance(res["neg"], ValueError)
    ws, wr = _direct(x, [3, 7], [1, 2], 300)
    s, r = res["good"]
    np.testing.assert_array_equal(r, wr)
    assert len(r) == 298
    assert sum(calls) == 1
    ca.close()
    cb.close()
    srv.close()
    b.close()
