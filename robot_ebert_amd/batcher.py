"""Request micro-batcher: coalesce concurrent recommendation requests into one
batched ``score_topk`` call.

The reference serves one user per call: FastAPI runs the sync handler ``get_user_recommendations``
(``src/backend/app/api/users.py:150-155``) on up to 40 anyio worker threads, each calling
``lib.get_user_recs`` (``lib.py:32-63``) with B = 1. On MI355X a 1-query screen wastes the chip, so
request threads hand their (liked rows, rated rows, k) to ONE dispatcher thread that waits at
most ``max_wait_ms`` for company, runs a single ``score_topk`` over up to ``max_batch`` users and
hands each caller its own slice. The dispatcher is the only thread that touches the GPU (and, for a
sharded catalog, the process group: RCCL communicators must not be used concurrently, SURVEY §8b
"Threading").

Per-request semantics are those of ``lib.get_user_recs``: a request without liked rows fails
with sklearn's ValueError (alone -- the rest of its batch is unaffected), results are
(scores float64, global rows int64) ordered (score desc, row asc).
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

_SENTINEL = object()


class RecBatcher:
    def __init__(self, catalog, max_batch: int = 4096, max_wait_ms: float = 2.0,
                 score_fn: Optional[Callable] = None) -> None:
        """catalog: the ``Catalog`` every request scores against. score_fn(catalog, k, liked=,
        exclude=) -> (scores [B, k], rows [B, k]) defaults to ``search.score_topk``."""
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        if score_fn is None:
            from .search import score_topk as score_fn
        self.catalog = catalog
        self.max_batch = int(max_batch)
        self.max_wait = float(max_wait_ms) / 1e3
        self._score = score_fn
        self._q: "queue.Queue" = queue.Queue()
        self._closed = False
        self._lock = threading.Lock()  # orders submit()'s check-and-put against close()
        self.batches: List[int] = []  # sizes of the batches run (observability / tests)
        self._thread = threading.Thread(target=self._run, name="ebert-batcher", daemon=True)
        self._thread.start()

    # ---- request side (any thread) -----------------------------------------------------------
    def submit(self, liked_rows: Sequence[int], exclude_rows: Sequence[int], k: int) -> Future:
        """Queue one user's request; the Future resolves to (scores [k'], rows [k']) numpy arrays
        (k' <= k: fewer when the catalog has fewer candidates) or raises the request's error."""
        fut: Future = Future()
        if k < 1:
            fut.set_exception(ValueError("k must be >= 1"))
            return fut
        if len(liked_rows) == 0:  # lib.py:51 with an empty X -> sklearn check_pairwise_arrays
            fut.set_exception(ValueError(
                f"Found array with 0 sample(s) (shape=(0, {self.catalog.d})) while a minimum of 1 "
                "is required by check_pairwise_arrays."))
            return fut
        item = (list(liked_rows), sorted(set(int(r) for r in exclude_rows)), int(k), fut)
        with self._lock:   # a request is either queued before close()'s sentinel or refused
            if self._closed:
                fut.set_exception(RuntimeError("batcher is closed"))
                return fut
            self._q.put(item)
        return fut

    def close(self, timeout: Optional[float] = 10.0) -> None:
        """Stop accepting requests, finish the queued ones, join the dispatcher."""
        with self._lock:
            if self._closed:
                return
            self._closed = True
            self._q.put(_SENTINEL)
        self._thread.join(timeout)

    # ---- dispatcher thread ---------------------------------------------------------------------
    def _collect(self) -> Tuple[list, bool]:
        first = self._q.get()
        if first is _SENTINEL:
            return [], True
        reqs = [first]
        deadline = time.monotonic() + self.max_wait
        stop = False
        while len(reqs) < self.max_batch:
            left = deadline - time.monotonic()
            try:
                item = self._q.get(timeout=max(left, 0.0)) if left > 0 else self._q.get_nowait()
            except queue.Empty:
                break
            if item is _SENTINEL:
                stop = True
                break
            reqs.append(item)
        return reqs, stop

    def _run(self) -> None:
        while True:
            reqs, stop = self._collect()
            if reqs:
                self._dispatch(reqs)
            if stop:
                while True:  # drain what was queued before close()
                    try:
                        item = self._q.get_nowait()
                    except queue.Empty:
                        return
                    if item is not _SENTINEL:
                        self._dispatch([item])

    def _dispatch(self, reqs: list) -> None:
        k_max = max(r[2] for r in reqs)
        try:
            scores, rows = self._score(self.catalog, k_max, liked=[r[0] for r in reqs],
                                       exclude=[r[1] for r in reqs])
            scores = scores.cpu().numpy() if hasattr(scores, "cpu") else np.asarray(scores)
            rows = rows.cpu().numpy() if hasattr(rows, "cpu") else np.asarray(rows)
        except BaseException as e:  # the whole batch failed: every caller sees the error
            for r in reqs:
                r[3].set_exception(e)
            return
        self.batches.append(len(reqs))
        for i, (_, _, k, fut) in enumerate(reqs):
            s, r = scores[i, :k], rows[i, :k]
            keep = r >= 0
            fut.set_result((s[keep], r[keep]))
