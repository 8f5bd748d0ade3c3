"""Request micro-batcher: coalesce concurrent recommendation requests into one
batched ``score_topk`` call.

The reference serves one user per call: FastAPI runs the sync handler ``get_user_recommendations``
(``src/backend/app/api/users.py:150-155``) on up to 40 anyio worker threads, each calling
``lib.get_user_recs`` (``lib.py:32-63``) with B = 1. On MI355X a 1-query screen wastes the chip, so
request threads hand their (liked rows, rated rows, k) to ONE dispatcher thread that waits at
most ``max_wait_ms`` for company, runs a single batched search over up to ``max_batch`` users and
hands each caller its own slice. Only the batcher's threads touch the GPU; with an injected
``score_fn`` (e.g. a sharded catalog's step, whose RCCL communicators must not be used
concurrently, SURVEY §8b "Threading") only the dispatcher does.

* k classes: a batch runs at the largest k among its requests, so requests are grouped by k class
  (``K_CLASSES``: the screen's k' and merge path change with k) and a large-k request does not pull
  small-k users onto the large-k path.
* Pipelining (default scoring): the dispatcher submits a batch (``search.score_topk_submit``: its
  kernels enqueued) and goes back to collecting; a completion thread finishes the batches in
  order (``score_topk_finish``: it waits in the C library, without the GIL) and answers their
  callers, so collection and GPU work overlap and no thread polls (under FastAPI's 40 request
  threads every wake-up competes for the GIL). At most ``max_inflight`` batches are submitted and
  not yet finished. With an injected ``score_fn`` the batch runs synchronously.
* Bounded statistics: ``batches`` keeps the sizes of the last ``history`` batches; ``stats()``
  gives totals and a power-of-two batch-size histogram.

Per-request semantics are those of ``lib.get_user_recs``: a request without liked rows fails
with sklearn's ValueError (alone -- the rest of its batch is unaffected), results are
(scores float64, global rows int64) ordered (score desc, row asc).
"""
from __future__ import annotations

import collections
import os
import queue
import threading
import time
from concurrent.futures import Future
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

_SENTINEL = object()
# requests with k in (K_CLASSES[i-1], K_CLASSES[i]] share a batch; the last class is unbounded
K_CLASSES = (32, 128, 512, 4096)


def _answer(fut: Future, result=None, exc: Optional[BaseException] = None) -> None:
    """Resolve a caller's Future unless it is already done (cancelled by its caller, or answered):
    one abandoned request must never stop the thread that answers the others."""
    if fut.done():
        return
    try:
        if exc is not None:
            fut.set_exception(exc)
        else:
            fut.set_result(result)
    except Exception:  # noqa: BLE001 -- InvalidStateError: cancelled in between
        pass


def k_class(k: int) -> int:
    for i, hi in enumerate(K_CLASSES):
        if k <= hi:
            return i
    return len(K_CLASSES)


class RecBatcher:
    def __init__(self, catalog, max_batch: int = 4096, max_wait_ms: float = 2.0,
                 score_fn: Optional[Callable] = None, history: int = 1024,
                 max_inflight: int = 2, stager="auto", submit_fn: Optional[Callable] = None,
                 finish_fn: Optional[Callable] = None,
                 stage_min_bytes: Optional[int] = None) -> None:
        """catalog: the ``Catalog`` every request scores against. score_fn(catalog, k, liked=,
        exclude=) -> (scores [B, k], rows [B, k]); default: ``search.score_topk_submit`` /
        ``score_topk_finish`` (or submit_fn / finish_fn) with up to ``max_inflight`` batches on
        the GPU. stager: the host boundary's copy stream (hostio.HostStager; "auto" = one on the
        catalog's GPU, None = copies in line): a batch's liked / rated CSR goes to the device
        under the previous batch's kernels and its results come back under the next one's --
        for batches whose CSRs reach `stage_min_bytes` (default 1 MiB, EBERT_STAGE_MIN_BYTES).
        A route-sized batch (tens of users, tens of KB) goes in line: its copies take
        microseconds, and the staging's dozen host-side stream / event / pinned-buffer calls per
        batch cost more than they hide (round 6, tools/route_bench.py with and without: batched
        scoring 10.1-11.0K requests/s staged vs 15.0-15.7K in line, profiles/r6/route/)."""
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.catalog = catalog
        self._submit_fn, self._finish_fn = submit_fn, finish_fn
        if stager == "auto":
            dev = getattr(catalog, "device", None)
            stager = None
            if (score_fn is None and dev is not None and getattr(dev, "type", None) == "cuda"
                    and os.environ.get("EBERT_HOST_STAGER", "1") != "0"):   # "0": A/B knob
                from .hostio import HostStager
                stager = HostStager(dev)
        self.stager = stager
        self.stage_min_bytes = int(stage_min_bytes if stage_min_bytes is not None
                                   else os.environ.get("EBERT_STAGE_MIN_BYTES", 1 << 20))
        self.max_batch = int(max_batch)
        self.max_wait = float(max_wait_ms) / 1e3
        self._score = score_fn
        self._pipelined = score_fn is None
        self.max_inflight = max(1, int(max_inflight))
        self._q: "queue.Queue" = queue.Queue()
        self._closed = False
        self._lock = threading.Lock()  # orders submit()'s check-and-put against close()
        self.batches = collections.deque(maxlen=int(history))  # sizes of the last batches
        self._n_batches = 0
        self._n_requests = 0
        self._hist: Dict[int, int] = collections.Counter()
        self._done: "queue.Queue" = queue.Queue()      # submitted batches, in order
        self._slots = threading.Semaphore(self.max_inflight)
        self._completer = None
        if self._pipelined:
            self._completer = threading.Thread(target=self._complete, name="ebert-batcher-done",
                                               daemon=True)
            self._completer.start()
        self._thread = threading.Thread(target=self._run, name="ebert-batcher", daemon=True)
        self._thread.start()

    # ---- request side (any thread) -----------------------------------------------------------
    def submit(self, liked_rows: Sequence[int], exclude_rows: Sequence[int], k: int) -> Future:
        """Queue one user's request; the Future resolves to (scores [k'], rows [k']) numpy arrays
        (k' <= k: fewer when the catalog has fewer candidates) or raises the request's error."""
        fut: Future = Future()
        # every request is checked HERE, before it can share a batch: the batch is one library
        # call, and an argument the library rejects (a liked row outside the catalog, a k whose
        # workspace cannot exist) would fail every co-batched request, other clients' included
        try:
            k = int(k)
            liked = [int(r) for r in liked_rows]
            rated = [int(r) for r in exclude_rows]
        except (TypeError, ValueError, OverflowError) as e:
            fut.set_exception(ValueError(f"malformed request: {e}"))
            return fut
        if k < 1:
            fut.set_exception(ValueError("k must be >= 1"))
            return fut
        if len(liked) == 0:  # lib.py:51 with an empty X -> sklearn check_pairwise_arrays
            fut.set_exception(ValueError(
                f"Found array with 0 sample(s) (shape=(0, {self.catalog.d})) while a minimum of 1 "
                "is required by check_pairwise_arrays."))
            return fut
        lo = int(getattr(self.catalog, "row_offset", 0))
        n = int(getattr(self.catalog, "n", 0))
        hi = lo + n
        if n > 0 and any(r < lo or r >= hi for r in liked):
            bad = next(r for r in liked if r < lo or r >= hi)
            fut.set_exception(ValueError(f"liked row {bad} is not in the catalog rows [{lo}, {hi})"))
            return fut
        # rated rows outside the catalog cannot match a candidate: dropped, as lib.py:48's
        # catalog.index.difference(rated) ignores unknown ids. k past the catalog returns every
        # candidate (the Future holds at most n rows): the same answer from a k the library can size
        if n > 0:
            rated = [r for r in rated if lo <= r < hi]
            k = min(k, int(getattr(self.catalog, "n_global", n)))
        item = (liked, sorted(set(rated)), k, fut)
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
        if self._completer is not None:
            self._completer.join(timeout)

    def stats(self) -> dict:
        """Totals since start and the batch-size histogram (bin b = sizes in [2^b, 2^(b+1)))."""
        return {"batches": self._n_batches, "requests": self._n_requests,
                "mean_batch": self._n_requests / max(self._n_batches, 1),
                "size_hist_pow2": dict(sorted(self._hist.items()))}

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
                item = self._q.get(timeout=left) if left > 0 else self._q.get_nowait()
            except queue.Empty:
                break
            if item is _SENTINEL:
                stop = True
                break
            reqs.append(item)
        return reqs, stop

    def _run(self) -> None:
        if self._pipelined:
            self._bind_device()
        while True:
            reqs, stop = self._collect()
            if reqs:
                groups: Dict[int, list] = collections.defaultdict(list)
                for r in reqs:
                    groups[k_class(r[2])].append(r)
                for c in sorted(groups):
                    self._dispatch_safe(groups[c])
            if stop:
                while True:  # drain what was queued before close()
                    try:
                        item = self._q.get_nowait()
                    except queue.Empty:
                        break
                    if item is not _SENTINEL:
                        self._dispatch_safe([item])
                self._done.put(_SENTINEL)
                return

    def _record(self, n: int) -> None:
        self.batches.append(n)
        self._n_batches += 1
        self._n_requests += n
        self._hist[max(n, 1).bit_length() - 1] += 1

    def _dispatch_safe(self, reqs: list) -> None:
        """_dispatch, and if anything in it fails unexpectedly, that error to every caller of the
        batch not answered yet: the dispatcher thread itself never dies with callers waiting."""
        try:
            self._dispatch(reqs)
        except BaseException as e:  # noqa: BLE001
            for r in reqs:
                _answer(r[3], exc=e)

    def _dispatch(self, reqs: list) -> None:
        k_max = max(r[2] for r in reqs)
        liked, excl = [r[0] for r in reqs], [r[1] for r in reqs]
        if not self._pipelined:
            try:
                scores, rows = self._score(self.catalog, k_max, liked=liked, exclude=excl)
            except BaseException as e:  # the whole batch failed: every caller sees the error
                for r in reqs:
                    _answer(r[3], exc=e)
                return
            self._deliver(reqs, scores, rows)
            return
        submit = self._submit_fn
        if submit is None:
            from .search import score_topk_submit as submit
        self._slots.acquire()            # released by the completion thread
        try:
            ev = None
            # the batch's CSR bytes (offsets + rows, liked and rated)
            nbytes = 8 * (2 * (len(liked) + 1) + sum(len(x) for x in liked) +
                          sum(len(x) for x in excl))
            if self.stager is not None and nbytes >= self.stage_min_bytes:
                # the batch's CSRs through the copy stream (pinned staging), then its kernels;
                # an event right after them for its results' D2H
                from .search import csr_from_lists
                dev = self.catalog.device
                liked = csr_from_lists(liked, dev, self.stager)
                excl = csr_from_lists(excl, dev, self.stager)
                p = submit(self.catalog, k_max, liked=liked, exclude=excl)
                ev = self.stager.record()
            else:
                p = submit(self.catalog, k_max, liked=liked, exclude=excl)
        except BaseException as e:
            self._slots.release()
            for r in reqs:
                _answer(r[3], exc=e)
            return
        self._done.put((p, reqs, ev))

    def _complete(self) -> None:
        """Completion thread: finish the submitted batches in order and answer their callers."""
        finish = self._finish_fn
        if finish is None:
            from .search import score_topk_finish as finish
        from .hostio import retried
        self._bind_device()
        while True:
            item = self._done.get()
            if item is _SENTINEL:
                return
            p, reqs, ev = item
            try:   # the slot is released whatever happens to this batch's callers
                try:
                    scores, rows = finish(p)
                    if ev is not None:
                        # D2H on the copy stream after this batch's kernels only (a fresh event
                        # when its retries ran behind later batches), under the next batch
                        if retried(p):
                            ev = self.stager.record()
                        scores, rows = self.stager.to_host((scores, rows), ev).result()
                except BaseException as e:  # noqa: BLE001
                    for r in reqs:
                        _answer(r[3], exc=e)
                    continue
                self._deliver(reqs, scores, rows)
            except BaseException as e:  # noqa: BLE001 -- never let one batch stop the thread
                for r in reqs:             # (its callers not answered yet get the error)
                    _answer(r[3], exc=e)
            finally:
                self._slots.release()

    def _bind_device(self) -> None:
        """Both batcher threads run on the catalog's device: libebert's per-device event pools
        key on the calling thread's current HIP device."""
        dev = getattr(self.catalog, "device", None)
        if dev is not None and getattr(dev, "type", None) == "cuda":
            import torch
            torch.cuda.set_device(dev)

    def _deliver(self, reqs: list, scores, rows) -> None:
        try:
            scores = scores.cpu().numpy() if hasattr(scores, "cpu") else np.asarray(scores)
            rows = rows.cpu().numpy() if hasattr(rows, "cpu") else np.asarray(rows)
        except BaseException as e:
            for r in reqs:
                _answer(r[3], exc=e)
            return
        self._record(len(reqs))
        for i, (_, _, k, fut) in enumerate(reqs):
            s, r = scores[i, :k], rows[i, :k]
            keep = r >= 0
            _answer(fut, (s[keep], r[keep]))
