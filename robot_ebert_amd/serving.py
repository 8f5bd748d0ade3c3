"""Multi-process serving of the recommend route.

The reference serves ``GET /users/{user_id}/recommendations/`` (``src/backend/app/api/users.py:
150-155``) from a sync handler on FastAPI's anyio worker threads; every request runs the ratings
SQL, the pandas filtering and the hydration (``lib.py:32-63``) under one interpreter lock. One
process's route is therefore bound by its Python host work (≈ 0.8 ms of GIL per request here),
not by the GPU, which scores a batch of thousands of users in milliseconds. So the route scales
the way the reference deploys it -- several server processes -- with ONE process owning the GPU:

* ``ScoreServer`` (the GPU-owning process): accepts connections from the server processes on a
  Unix socket; one reader thread per connection turns each request frame into a
  ``batcher.RecBatcher`` submission, so requests of every process are coalesced into one batched
  ``score_topk`` (the batcher's k classes, pipelining and per-request errors), and the answer goes
  back on the same connection as soon as its batch finishes.
* ``ScoreClient`` (each server process): thread-safe; one connection per process multiplexed by
  request id (a reader thread resolves each caller's Future), so a worker thread waits for its
  answer without holding the GIL.
* ``CatalogIndex``: the catalog's id index without the GPU (``Catalog.index_pos`` / ``rows_of`` /
  ``id_of``), what ``lib._user_request`` and ``lib._hydrate`` need in a server process.

Wire format (little-endian; one frame per ``Connection.send_bytes``):
  request  ``<QiII`` (request id, k, liked count L, rated count R) + L + R int64 global rows;
  response ``<QiI`` (request id, status, n) + n float64 scores + n int64 rows (status 0), or the
           UTF-8 text ``"<ExceptionType>: <message>"`` (status 1: ValueError / RuntimeError /
           KeyError are re-raised with that type in the caller, anything else as RuntimeError).
Per-request semantics are the batcher's, i.e. ``lib.get_user_recs``'s.
"""
from __future__ import annotations

import itertools
import os
import queue
import struct
import threading
from concurrent.futures import Future
from multiprocessing.connection import Client, Listener
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

_REQ = struct.Struct("<QiII")
_RESP = struct.Struct("<QiI")
_ERRORS = {"ValueError": ValueError, "RuntimeError": RuntimeError, "KeyError": KeyError}
AUTHKEY = b"robot-ebert-amd"


class CatalogIndex:
    """The string-id index of a catalog (the DataFrame index of constants.py:56) without its
    embeddings: ``index_pos`` / ``contains`` / ``rows_of`` / ``id_of`` exactly as ``Catalog``'s, and
    ``d`` (sklearn's error text of a user without liked movies quotes it)."""

    def __init__(self, ids: Sequence[str], d: int, row_offset: int = 0) -> None:
        self.ids: List[str] = list(ids)
        self.n, self.d, self.row_offset = len(self.ids), int(d), int(row_offset)
        self._pos: Optional[Dict[str, int]] = None

    @property
    def index_pos(self) -> Dict[str, int]:
        if self._pos is None:
            self._pos = {t: i for i, t in enumerate(self.ids)}
        return self._pos

    def contains(self, tmdb_ids: Iterable[str]) -> List[bool]:
        pos = self.index_pos
        return [t in pos for t in tmdb_ids]

    def rows_of(self, tmdb_ids: Iterable[str]) -> List[int]:
        pos = self.index_pos
        return [pos[t] + self.row_offset for t in tmdb_ids]

    def id_of(self, global_row: int) -> str:
        return self.ids[global_row - self.row_offset]


def encode_request(rid: int, liked: Sequence[int], rated: Sequence[int], k: int) -> bytes:
    lk = np.asarray(liked, dtype="<i8")
    rt = np.asarray(rated, dtype="<i8")
    return _REQ.pack(rid, int(k), lk.size, rt.size) + lk.tobytes() + rt.tobytes()


def decode_request(buf: bytes) -> Tuple[int, int, np.ndarray, np.ndarray]:
    rid, k, nl, nr = _REQ.unpack_from(buf, 0)
    o = _REQ.size
    if len(buf) != o + 8 * (nl + nr):
        raise ValueError(f"malformed request frame ({len(buf)} bytes for {nl} + {nr} rows)")
    lk = np.frombuffer(buf, dtype="<i8", count=nl, offset=o)
    rt = np.frombuffer(buf, dtype="<i8", count=nr, offset=o + 8 * nl)
    return rid, k, lk, rt


def encode_response(rid: int, scores=None, rows=None, exc: Optional[BaseException] = None) -> bytes:
    if exc is not None:
        msg = f"{type(exc).__name__}: {exc}".encode("utf-8", errors="replace")
        return _RESP.pack(rid, 1, len(msg)) + msg
    s = np.ascontiguousarray(scores, dtype="<f8")
    r = np.ascontiguousarray(rows, dtype="<i8")
    return _RESP.pack(rid, 0, s.size) + s.tobytes() + r.tobytes()


def decode_response(buf: bytes):
    """(request id, (scores, rows)) or (request id, exception)."""
    rid, status, n = _RESP.unpack_from(buf, 0)
    o = _RESP.size
    if status != 0:
        text = bytes(buf[o:o + n]).decode("utf-8", errors="replace")
        name, _, msg = text.partition(": ")
        if name == "KeyError":
            msg = msg.strip("'")
        return rid, _ERRORS.get(name, RuntimeError)(msg if name in _ERRORS else text)
    s = np.frombuffer(buf, dtype="<f8", count=n, offset=o).copy()
    r = np.frombuffer(buf, dtype="<i8", count=n, offset=o + 8 * n).copy()
    return rid, (s, r)


def _shutdown(conn) -> None:
    """Shut a Connection's socket down in both directions: a thread blocked in recv_bytes on it
    (here or at the peer) sees EOF. The fd itself is closed by its reader."""
    import socket
    try:
        s = socket.socket(fileno=os.dup(conn.fileno()))
        try:
            s.shutdown(socket.SHUT_RDWR)
        finally:
            s.close()
    except OSError:
        pass


class ScoreServer:
    """The GPU-owning side: requests from any number of client connections go to one
    ``RecBatcher`` (or anything with its ``submit(liked, rated, k) -> Future``)."""

    def __init__(self, batcher, address: Optional[str] = None) -> None:
        self.batcher = batcher
        self.address = address or os.path.join(
            "/tmp", f"ebert-score-{os.getpid()}-{id(self):x}.sock")
        self._listener = Listener(self.address, family="AF_UNIX", authkey=AUTHKEY)
        try:   # this user's processes only (the handshake key is not a secret)
            os.chmod(self.address, 0o600)
        except OSError:
            pass
        self._closed = False
        self._conns: list = []
        self._lock = threading.Lock()
        self.requests = 0              # frames received (a statistic; updated without a lock)
        self._accept = threading.Thread(target=self._accept_loop, name="ebert-score-accept",
                                        daemon=True)
        self._accept.start()

    def _accept_loop(self) -> None:
        while not self._closed:
            try:
                conn = self._listener.accept()
            except (OSError, EOFError):
                if self._closed:
                    return
                continue
            except Exception:  # noqa: BLE001 -- a client failing the handshake
                continue
            with self._lock:
                if self._closed:
                    _shutdown(conn)
                    conn.close()
                    return
                self._conns.append(conn)
            threading.Thread(target=self._serve, args=(conn,), name="ebert-score-conn",
                             daemon=True).start()

    def _serve(self, conn) -> None:
        # answers go out through this connection's writer thread: the batcher's completion
        # thread only queues a frame, so a client that stops reading (a full socket buffer)
        # blocks its own writer, never the batcher and the other connections
        outq: "queue.SimpleQueue[Optional[bytes]]" = queue.SimpleQueue()

        def write_loop() -> None:
            while True:
                frame = outq.get()
                if frame is None:
                    return
                try:
                    conn.send_bytes(frame)
                except (OSError, EOFError, ValueError):
                    # the client went away: drop its answers, wake its reader
                    _shutdown(conn)
                    while outq.get() is not None:
                        pass
                    return
        writer = threading.Thread(target=write_loop, name="ebert-score-write", daemon=True)
        writer.start()
        reply = outq.put

        while True:
            try:
                buf = conn.recv_bytes()
            except (OSError, EOFError):
                break
            try:
                rid, k, liked, rated = decode_request(buf)
            except Exception as e:  # noqa: BLE001 -- a malformed frame ends the connection
                reply(encode_response(0, exc=e))
                break
            self.requests += 1
            fut = self.batcher.submit(liked.tolist(), rated.tolist(), k)

            def done(f: Future, rid=rid) -> None:
                e = f.exception()
                if e is not None:
                    reply(encode_response(rid, exc=e))
                else:
                    s, r = f.result()
                    reply(encode_response(rid, s, r))
            fut.add_done_callback(done)
        with self._lock:
            if conn in self._conns:
                self._conns.remove(conn)
        # answers still pending in the batcher are queued after the sentinel and dropped; the
        # writer sends what was queued before it (an error reply of a malformed frame included)
        outq.put(None)
        writer.join(5.0)
        try:
            conn.close()
        except OSError:
            pass

    def close(self) -> None:
        """Stop accepting, close every connection (the batcher stays the caller's)."""
        with self._lock:
            if self._closed:
                return
            self._closed = True
        # wake the accept thread (blocked in accept(): closing the socket does not) with a bare
        # connect: its handshake fails there, and nothing here waits for it (the thread may
        # already have seen the flag and ended)
        import socket
        try:
            with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as w:
                w.settimeout(1.0)
                w.connect(self.address)
        except OSError:
            pass
        self._accept.join(5.0)
        try:
            self._listener.close()
        except OSError:
            pass
        with self._lock:   # no connection is registered after the accept thread has ended
            conns, self._conns = list(self._conns), []
        for c in conns:   # shutdown wakes the connection's reader blocked in recv (close does not)
            _shutdown(c)
        try:
            os.unlink(self.address)
        except OSError:
            pass


class ScoreClient:
    """A server process's connection to the ``ScoreServer``: ``submit`` from any thread; answers
    come back in any order and resolve the callers' Futures (a reader thread)."""

    def __init__(self, address: str, timeout: float = 60.0) -> None:
        self._conn = Client(address, family="AF_UNIX", authkey=AUTHKEY)
        self._send = threading.Lock()
        self._pending: Dict[int, Future] = {}
        self._plock = threading.Lock()
        self._ids = itertools.count(1)
        self._closed = False
        self.timeout = timeout
        self._reader = threading.Thread(target=self._read_loop, name="ebert-score-client",
                                        daemon=True)
        self._reader.start()

    def _read_loop(self) -> None:
        err: BaseException = RuntimeError("score server connection closed")
        while True:
            try:
                buf = self._conn.recv_bytes()
            except (OSError, EOFError) as e:
                err = RuntimeError(f"score server connection closed ({e!r})")
                break
            try:
                rid, res = decode_response(buf)
            except Exception as e:  # noqa: BLE001 -- a garbled frame: the stream is unusable
                err = RuntimeError(f"score server sent a malformed frame ({e!r})")
                _shutdown(self._conn)
                break
            with self._plock:
                fut = self._pending.pop(rid, None)
            if fut is None or not fut.set_running_or_notify_cancel():
                continue   # unknown id, or the caller cancelled its Future: drop the answer
            if isinstance(res, BaseException):
                fut.set_exception(res)
            else:
                fut.set_result(res)
        with self._plock:
            left, self._pending = list(self._pending.values()), {}
            self._closed = True
        for f in left:
            if f.set_running_or_notify_cancel():
                f.set_exception(err)

    def submit(self, liked: Sequence[int], rated: Sequence[int], k: int) -> Future:
        """``RecBatcher.submit``'s interface: a Future of (scores float64 [k'], global rows int64
        [k']) of one user, or of the request's error (``lib.get_user_recs_batched`` takes either)."""
        fut: Future = Future()
        rid = next(self._ids)
        with self._plock:
            if self._closed:
                fut.set_exception(RuntimeError("score server connection closed"))
                return fut
            self._pending[rid] = fut
        frame = encode_request(rid, liked, rated, k)
        try:
            with self._send:
                self._conn.send_bytes(frame)
        except (OSError, ValueError) as e:
            with self._plock:
                mine = self._pending.pop(rid, None) is not None
            # (else the reader, ending on the same closed connection, already failed it)
            if mine and fut.set_running_or_notify_cancel():
                fut.set_exception(RuntimeError(f"score server connection failed ({e!r})"))
        return fut

    def score(self, liked: Sequence[int], rated: Sequence[int], k: int):
        """``submit(...).result()`` with the client's timeout."""
        return self.submit(liked, rated, k).result(timeout=self.timeout)

    def close(self) -> None:
        _shutdown(self._conn)
        self._reader.join(5.0)
        try:
            self._conn.close()
        except OSError:
            pass
