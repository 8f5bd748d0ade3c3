"""CPU: the request micro-batcher (§8f-2) and the ingest helpers (§8f-3), host logic only.

The batcher's scoring function is injected: here the float64 oracle (test infrastructure)
stands in for the GPU ``score_topk`` so the coalescing, per-request slicing, error isolation and
shutdown logic run without a GPU. The GPU path is covered in test_gpu_parity.py.
"""
import concurrent.futures as cf
import threading

import numpy as np
import pandas as pd
import pytest

from oracle import restatement as R
from robot_ebert_amd.batcher import RecBatcher
from robot_ebert_amd import ingest


class _Cat:
    def __init__(self, x):
        self.x, self.d = x, x.shape[1]


def _oracle_score(calls):
    def score(cat, k, liked, exclude):
        calls.append(len(liked))
        qs = np.stack([R.mean_cosine_query(cat.x[l]) for l in liked])
        return R.cosine_topk(qs, cat.x, k, exclude)
    return score


def _direct(cat, liked, excl, k):
    s, r = R.cosine_topk(R.mean_cosine_query(cat.x[liked])[None, :], cat.x, k, [excl])
    keep = r[0] >= 0
    return s[0][keep], r[0][keep]


def test_batcher_coalesces_and_slices():
    rng = np.random.default_rng(0)
    cat = _Cat(rng.standard_normal((500, 16)))
    calls = []
    b = RecBatcher(cat, max_batch=32, max_wait_ms=50.0, score_fn=_oracle_score(calls))
    reqs = [(list(rng.choice(500, 3, replace=False)), list(rng.choice(500, 20, replace=False)),
             int(k)) for k in rng.integers(1, 40, 40)]
    with cf.ThreadPoolExecutor(16) as ex:
        futs = list(ex.map(lambda r: b.submit(*r), reqs))
        res = [f.result(timeout=30) for f in futs]
    b.close()
    for (liked, excl, k), (s, r) in zip(reqs, res):
        ws, wr = _direct(cat, liked, excl, k)
        np.testing.assert_array_equal(r, wr)
        np.testing.assert_allclose(s, ws, atol=1e-15)
    assert sum(calls) == len(reqs) and max(calls) > 1 and max(calls) <= 32


def test_batcher_errors_are_per_request():
    cat = _Cat(np.random.default_rng(1).standard_normal((50, 8)))
    b = RecBatcher(cat, max_batch=8, max_wait_ms=5.0, score_fn=_oracle_score([]))
    bad = b.submit([], [1, 2], 5)
    good = b.submit([3], [], 5)
    with pytest.raises(ValueError, match="0 sample"):
        bad.result(timeout=10)
    s, r = good.result(timeout=10)
    assert len(r) == 5
    b.close()
    assert isinstance(b.submit([1], [], 3).exception(timeout=1), RuntimeError)


def test_batcher_batch_failure_reaches_every_caller():
    def boom(cat, k, liked, exclude):
        raise MemoryError("out of HBM")
    b = RecBatcher(_Cat(np.zeros((4, 2))), max_batch=4, max_wait_ms=50.0, score_fn=boom)
    fs = [b.submit([0], [], 1) for _ in range(3)]
    for f in fs:
        assert isinstance(f.exception(timeout=10), MemoryError)
    b.close()


def test_ingest_chroma_matrix_and_id_order():
    ids = ["862", "10", "2", "1000", "99"]
    emb = np.arange(15, dtype=np.float32).reshape(5, 3)
    got_ids, m = ingest.chroma_matrix({"ids": ids, "embeddings": emb.tolist(), "documents": None})
    assert got_ids == ids and m.dtype == np.float64
    np.testing.assert_array_equal(m, emb)
    # lexicographic, as pandas sort_index on the str index of constants.py:56
    df = pd.DataFrame(m, index=ids)
    assert [ids[i] for i in ingest.id_order(ids)] == list(df.sort_index().index)
    with pytest.raises(Exception):
        ingest.chroma_matrix({"ids": ids[:4], "embeddings": emb.tolist()})
    with pytest.raises(Exception):
        ingest.chroma_matrix({"ids": ["a", "a"], "embeddings": [[1.0], [2.0]]})


def test_submit_racing_close_never_hangs():
    """a submit() racing close() is either served or refused -- never left queued
    behind the sentinel with a Future that does not resolve."""
    x = np.random.default_rng(9).standard_normal((300, 8))
    for trial in range(20):
        b = RecBatcher(_Cat(x), max_batch=4, max_wait_ms=0.5, score_fn=_oracle_score([]))
        futs = []
        start = threading.Event()

        def worker():
            start.wait()
            for i in range(25):
                futs.append(b.submit([i % 300], [], 3))
        ts = [threading.Thread(target=worker) for _ in range(4)]
        for t in ts:
            t.start()
        start.set()
        b.close()
        for t in ts:
            t.join()
        for f in futs:
            try:
                f.result(timeout=10)
            except RuntimeError as e:
                assert "closed" in str(e)


def test_batcher_groups_by_k_class():
    """A large-k request does not pull small-k users onto the large-k path: every batch holds
    one k class (batcher.K_CLASSES), and each caller still gets its own k."""
    from robot_ebert_amd.batcher import k_class
    rng = np.random.default_rng(5)
    cat = _Cat(rng.standard_normal((3000, 8)))
    seen = []

    def score(c, k, liked, exclude):
        seen.append(k)
        qs = np.stack([R.mean_cosine_query(c.x[l]) for l in liked])
        return R.cosine_topk(qs, c.x, k, exclude)
    b = RecBatcher(cat, max_batch=64, max_wait_ms=100.0, score_fn=score)
    ks = [5, 2000, 7, 100, 3, 2000, 30, 600]
    futs = [b.submit([i], [], k) for i, k in enumerate(ks)]
    res = [f.result(timeout=30) for f in futs]
    b.close()
    assert sorted(k_class(k) for k in seen) == sorted(set(k_class(k) for k in ks))
    assert max(seen) == 2000 and min(seen) == 30   # class 0 ran at its own k_max
    for (s, r), k in zip(res, ks):
        assert len(r) == k


def test_batcher_stats_are_bounded():
    cat = _Cat(np.random.default_rng(6).standard_normal((200, 8)))
    b = RecBatcher(cat, max_batch=4, max_wait_ms=0.0, score_fn=_oracle_score([]), history=4)
    for i in range(10):
        b.submit([i], [], 3).result(timeout=10)
    b.close()
    st = b.stats()
    assert len(b.batches) == 4 and st["batches"] == 10 and st["requests"] == 10
    assert sum(st["size_hist_pow2"].values()) == 10 and st["size_hist_pow2"] == {0: 10}


def test_pipelined_cancelled_request_does_not_wedge(monkeypatch):
    """in pipelined mode a caller that cancels its Future while its batch is
    on the GPU must not stop the completion thread (which would keep the in-flight slot and hang
    every later request). The GPU submit / finish pair is replaced by the float64 oracle here."""
    import robot_ebert_amd.search as S
    x = np.random.default_rng(11).standard_normal((400, 8))
    cat = _Cat(x)
    gate = threading.Event()

    def submit(c, k, liked, exclude):
        qs = np.stack([R.mean_cosine_query(c.x[l]) for l in liked])
        return R.cosine_topk(qs, c.x, k, exclude)

    def finish(p):
        gate.wait(10)
        return p
    monkeypatch.setattr(S, "score_topk_submit", submit)
    monkeypatch.setattr(S, "score_topk_finish", finish)
    b = RecBatcher(cat, max_batch=8, max_wait_ms=0.0, max_inflight=1)
    first = b.submit([1, 2], [3], 5)
    assert first.cancel()          # still pending: its batch waits in finish()
    gate.set()
    for i in range(6):             # one slot: every later batch needs the first one's release
        s, r = b.submit([i], [], 4).result(timeout=10)
        ws, wr = _direct(cat, [i], [], 4)
        np.testing.assert_array_equal(r, wr)
    b.close()
    assert b.stats()["requests"] >= 6


@pytest.mark.parametrize("pipelined", [False, True])
def test_batcher_malformed_result_fails_callers_not_thread(monkeypatch, pipelined):
    """A scoring function that returns something the delivery cannot slice (a bug, not a
    request's error): the batch's callers get that error and the batcher keeps serving."""
    import robot_ebert_amd.search as S
    x = np.random.default_rng(12).standard_normal((300, 8))
    cat = _Cat(x)
    bad = {"on": True}

    def score(c, k, liked, exclude):
        if bad["on"]:
            bad["on"] = False
            return np.zeros(3), None          # not (scores [B, k], rows [B, k])
        qs = np.stack([R.mean_cosine_query(c.x[l]) for l in liked])
        return R.cosine_topk(qs, c.x, k, exclude)
    if pipelined:
        monkeypatch.setattr(S, "score_topk_submit", score)
        monkeypatch.setattr(S, "score_topk_finish", lambda p: p)
        b = RecBatcher(cat, max_batch=4, max_wait_ms=0.0, max_inflight=1)
    else:
        b = RecBatcher(cat, max_batch=4, max_wait_ms=0.0, score_fn=score)
    first = b.submit([1], [], 3)
    assert first.exception(timeout=10) is not None
    for i in range(4):
        s, r = b.submit([i + 2], [], 3).result(timeout=10)
        np.testing.assert_array_equal(r, _direct(cat, [i + 2], [], 3)[1])
    b.close()
