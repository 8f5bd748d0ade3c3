"""CPU: the overlapped host boundary's ordering (robot_ebert_amd/hostio.py).

A recording stager stands in for the HIP copy stream: every H2D, event record and D2H is logged
with what it waits for. Checked, for the bench's pipeline (hostio.run_pipelined) and for the
request batcher's two threads (RecBatcher with a stager): batch i+1's H2D and submit are enqueued
before batch i is finished (so they run under batch i's kernels), batch i's D2H waits for the
event recorded right after batch i's own kernels (not for the stream's later work: batch i+1's),
a batch whose finish ran retries waits for a fresh event after them instead, and every answer
comes back to its own caller, equal to the float64 oracle (tests only; oracle/restatement.py).
"""
import threading

import numpy as np
import torch

from oracle import restatement as R
from robot_ebert_amd.batcher import RecBatcher
from robot_ebert_amd.hostio import run_pipelined


class Ev:
    def __init__(self, n):
        self.n = n


class Handle:
    def __init__(self, res):
        self.res = res

    def result(self):
        return tuple(np.asarray(x) for x in self.res)


class RecordingStager:
    def __init__(self):
        self.log = []
        self.threads = []     # the logging thread of each entry
        self.n = 0
        self.lock = threading.Lock()

    def add(self, e):
        with self.lock:
            self.log.append(e)
            self.threads.append(threading.current_thread().name)

    def to_device(self, x):
        self.add(("h2d", tag_of(x)))
        return torch.from_numpy(np.array(x, copy=True)) if isinstance(x, np.ndarray) else x

    def record(self):
        with self.lock:
            self.n += 1
            n = self.n
        self.add(("record", n))
        return Ev(n)

    def to_host(self, res, after):
        self.add(("d2h", res[0], after.n))
        return Handle(res[1:])


def tag_of(x):
    return x if isinstance(x, int) else "csr"


def test_run_pipelined_order():
    st = RecordingStager()
    log = st.log
    done = {}

    class P:
        def __init__(self, i):
            self.i = i

    def submit(d):
        st.add(("submit", d))
        return P(d)

    def finish(p):
        st.add(("finish", p.i))
        return (p.i, np.array([p.i]))

    res = [h.result() for h in run_pipelined(st, range(5), submit, finish,
                                              is_retried=lambda p: p.i == 2)]
    assert [int(r[0][0]) for r in res] == list(range(5))   # in order, each its own
    idx = {e: j for j, e in enumerate(log)}
    rec_after_submit = {}
    for j, e in enumerate(log):
        if e[0] == "submit":
            assert log[j + 1][0] == "record"             # the event right after its kernels
            rec_after_submit[e[1]] = log[j + 1][1]
    for i in range(1, 5):
        assert idx[("h2d", i)] < idx[("finish", i - 1)]
        assert idx[("submit", i)] < idx[("finish", i - 1)]
    d2h = {e[1]: e[2] for e in log if e[0] == "d2h"}
    for i in range(5):
        if i == 2:   # retried: a fresh event after its finish, later than batch 3's
            assert d2h[i] > rec_after_submit[3]
            j = idx[("finish", 2)]
            assert log[j + 1] == ("record", d2h[i])
        else:
            assert d2h[i] == rec_after_submit[i]
        done[i] = True
    assert len(done) == 5


def test_batcher_two_streams_order_and_answers():
    """RecBatcher with a stager: per batch the liked and rated CSRs go through to_device (the
    copy stream), the submit follows, then an event; the completion thread's D2H of that batch
    waits for exactly that event (or a fresh one after retries); answers equal the oracle."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((400, 12))

    class Cat:
        n, n_global, row_offset, d = 400, 400, 0, 12
        device = torch.device("cpu")

    st = RecordingStager()
    batches = []
    lock = threading.Lock()

    class P:
        def __init__(self, b, s, r, retry):
            self.b, self.s, self.r = b, s, r
            self.cert_host = torch.tensor([0 if retry else 1] * s.shape[0], dtype=torch.int32)

    def submit(cat, k, liked, exclude):
        lo, lr = liked
        eo, er = exclude
        lo, lr, eo, er = (t.numpy() for t in (lo, lr, eo, er))
        B = len(lo) - 1
        ls = [lr[lo[i]:lo[i + 1]].tolist() for i in range(B)]
        es = [er[eo[i]:eo[i + 1]].tolist() for i in range(B)]
        qs = np.stack([R.mean_cosine_query(x[l]) for l in ls])
        s, r = R.cosine_topk(qs, x, k, es)
        with lock:
            b = len(batches)
            batches.append(B)
        st.add(("submit", b))
        return P(b, s, r, retry=(b == 1))

    tag = {}

    def finish(p):
        st.add(("finish", p.b))
        tag[id(p.s)] = p.b
        return p.s, p.r

    # the batcher hands (scores, rows) to to_host: log them under their batch
    real_to_host = st.to_host

    def to_host(res, after):
        return real_to_host((tag[id(res[0])], *res), after)
    st.to_host = to_host

    b = RecBatcher(Cat(), max_batch=16, max_wait_ms=30.0, stager=st, submit_fn=submit,
                   finish_fn=lambda p: finish(p), stage_min_bytes=0)   # stage every batch
    reqs = [(sorted(rng.choice(400, 3, replace=False).tolist()),
             sorted(rng.choice(400, 5, replace=False).tolist()), int(k))
            for k in rng.integers(1, 20, 40)]
    futs = [b.submit(*q) for q in reqs]
    out = [f.result(timeout=30) for f in futs]
    b.close()
    for (liked, excl, k), (s, r) in zip(reqs, out):
        ws, wr = R.cosine_topk(R.mean_cosine_query(x[liked])[None, :], x, k, [excl])
        keep = wr[0] >= 0
        np.testing.assert_array_equal(r, wr[0][keep])
        np.testing.assert_allclose(s, ws[0][keep], rtol=0, atol=1e-15)
    assert len(batches) >= 2 and sum(batches) == len(reqs)
    # the dispatcher thread's own sequence (the completion thread logs concurrently)
    log = [e for e, t in zip(st.log, st.threads) if t == "ebert-batcher"]
    for j, e in enumerate(log):
        if e[0] == "submit":
            # two CSR copies (liked, rated) right before it, the event right after it
            assert log[j - 1] == ("h2d", "csr") and log[j - 2] == ("h2d", "csr")
            assert log[j + 1][0] == "record"
    ev_of = {log[j][1]: log[j + 1][1] for j in range(len(log)) if log[j][0] == "submit"}
    log = st.log
    for e in log:
        if e[0] == "d2h":
            bi, after = e[1], e[2]
            if bi == 1:   # its finish ran retries: a fresh event, after that finish
                f = log.index(("finish", 1))
                assert after > ev_of[1] and ("record", after) in log[f:]
            else:
                assert after == ev_of[bi]


def test_sorted_csr_host_facts_and_retried():
    """csr_from_lists' SortedCSR carries the host facts that let the C entry skip reading the
    liked CSR back (EBT_FLAG_LIKED_CHECKED only when every segment is non-empty and every row in
    the catalog's range); hostio.retried reads a finished batch's first-pass certificates (and
    the C entry's k > n padding) to decide whether its results' D2H needs a fresh event."""
    from robot_ebert_amd.hostio import retried
    from robot_ebert_amd.search import SortedCSR, csr_from_lists, csr_sorted
    c = csr_from_lists([[5, 1, 3], [7], [2, 2]], torch.device("cpu"))
    assert isinstance(c, SortedCSR) and c.min_len == 1 and (c.row_min, c.row_max) == (1, 7)
    assert c[0].tolist() == [0, 3, 4, 6] and c[1].tolist() == [1, 3, 5, 7, 2, 2]
    assert c.checked_for(0, 8) and not c.checked_for(0, 7) and not c.checked_for(2, 100)
    e = csr_from_lists([[4], []], torch.device("cpu"))
    assert e.min_len == 0 and not e.checked_for(0, 100)
    z = csr_from_lists([[], []], torch.device("cpu"))
    assert z.row_min is None and not z.checked_for(0, 100)
    assert not SortedCSR(c[0], c[1]).checked_for(0, 100)   # facts unknown: not checked
    assert csr_sorted(c) is c

    class Rec:
        def __init__(self, B, k, k_eff):
            self.B, self.k, self.k_eff = B, k, k_eff

    class P:
        def __init__(self, cert, rec=None):
            self.cert_host = torch.tensor(cert, dtype=torch.int32)
            if rec is not None:
                self.pending = rec
    assert not retried(P([1, 1, 1, 77], Rec(3, 10, 10)))    # slot B is the C entry's flag
    assert retried(P([1, 0, 1, 0], Rec(3, 10, 10)))
    assert retried(P([1, 1, 1, 0], Rec(3, 10, 5)))          # k > n: padded in the finish
    assert not retried(P([1, 1]))                           # the Python path: B entries
    assert retried(P([1, -1]))
    assert retried(object())                                # unknown: a fresh event


def test_batcher_small_batches_go_in_line():
    """Below stage_min_bytes (default 1 MiB of CSR) a batch's copies go in line, no staging:
    route-sized batches pay the staging's host calls without anything to hide
    (profiles/r6/route/: batched scoring 10.1-11.0K requests/s staged vs 15.0-15.7K in line)."""
    rng = np.random.default_rng(4)
    x = rng.standard_normal((300, 8))

    class Cat:
        n, n_global, row_offset, d = 300, 300, 0, 8
        device = torch.device("cpu")

    st = RecordingStager()

    class P:
        def __init__(self, s, r):
            self.s, self.r = s, r
            self.cert_host = torch.ones(s.shape[0], dtype=torch.int32)

    def submit(cat, k, liked, exclude):
        assert isinstance(liked, list)     # host lists: the C path builds the CSR in line
        qs = np.stack([R.mean_cosine_query(x[l]) for l in liked])
        return P(*R.cosine_topk(qs, x, k, exclude))
    b = RecBatcher(Cat(), max_batch=8, max_wait_ms=20.0, stager=st, submit_fn=submit,
                   finish_fn=lambda p: (p.s, p.r))
    assert b.stage_min_bytes == 1 << 20
    out = [b.submit([i, i + 1], [i + 2], 5) for i in range(20)]
    for f in out:
        s, r = f.result(timeout=30)
        assert len(r) == 5
    b.close()
    assert st.log == []
