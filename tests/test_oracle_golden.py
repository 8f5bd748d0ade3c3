"""CPU: pin the float64 oracle restatement against the reference's own outputs.

The vectors in tests/golden/ were produced by importing the reference's get_user_recs / run_search
(tests/golden/make_golden.py) and by the sklearn + pandas calls the reference makes.
"""
import json
import os

import numpy as np
import pytest

from inputs import COS_CASES, c1_catalog, cos_case_inputs, sha256_array
from oracle import restatement as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def c1():
    with open(os.path.join(GOLD, "c1_collab.json")) as f:
        return json.load(f)


def test_c1_inputs_regenerate(c1):
    ids, cat = c1_catalog()
    assert sha256_array(cat) == c1["catalog_sha256"]
    assert len(ids) == 2269 and ids == sorted(ids)


@pytest.mark.parametrize("k", [10, 10000])
def test_c1_get_user_recs_matches_reference(c1, k):
    ids, cat = c1_catalog()
    for uid, rec in c1["users"].items():
        want = rec[f"k{k}"]
        ratings = [tuple(x) for x in rec["ratings"]]
        if isinstance(want, dict):
            with pytest.raises(ValueError) as ei:
                R.get_user_recs(ratings, ids, cat, k)
            assert str(ei.value) == want["message"]
            continue
        got = R.get_user_recs(ratings, ids, cat, k)
        assert [g[0] for g in got] == [w[0] for w in want], uid
        np.testing.assert_allclose([g[1] for g in got], [w[1] for w in want], rtol=0, atol=1e-12)


def test_c1_edge_cases_present(c1):
    u = c1["users"]
    assert u["u00"]["k10"] == []                                   # no ratings
    assert u["u01"]["k10"]["error"] == "ValueError"                # no liked movie
    assert len(u["u04"]["k10000"]) == 2269 - 5                     # k > candidates
    assert any(t == "999999999" for t, _ in u["u02"]["ratings"])   # id not in catalog


def test_search_reweight_matches_reference(c1):
    ids, cat = c1_catalog()
    s = c1["search"]
    pos = {t: i for i, t in enumerate(ids)}
    mids, msc = s["match_ids"], np.array(s["match_scores"])
    for uid, want in s["cases"].items():
        if isinstance(want, dict):
            continue
        if uid == "None":
            pop = np.array(s["popularity"])
            user = (pop - pop.min()) / (pop.max() - pop.min())
        else:
            ratings = c1["users"][uid]["ratings"]
            liked = [pos[t] for t, r in ratings if t in pos and r >= 3.5]
            user = R.cosine_similarity(cat[liked], cat[[pos[m] for m in mids]]).mean(axis=0)
        comb = R.reweight_scores(msc, user)
        order = sorted(range(len(mids)), key=lambda i: -comb[i])
        assert [mids[i] for i in order] == [w[0] for w in want]
        np.testing.assert_allclose([comb[i] for i in order], [w[1] for w in want], atol=1e-12)


@pytest.mark.parametrize("name", sorted(COS_CASES))
def test_cos_topk_matches_sklearn_pandas(name):
    case = COS_CASES[name]
    with open(os.path.join(GOLD, "cos_topk_small.json")) as f:
        meta = json.load(f)[name]
    gold = np.load(os.path.join(GOLD, "cos_topk_small.npz"))
    q, c, excl = cos_case_inputs(case)
    assert sha256_array(q) == meta["q_sha256"] and sha256_array(c) == meta["c_sha256"]
    s, r = R.cosine_topk(q, c, case["k"], excl)
    np.testing.assert_array_equal(r, gold[f"{name}_rows"])
    np.testing.assert_allclose(s, gold[f"{name}_scores"], rtol=0, atol=1e-12)


def test_merge_equals_unsharded():
    case = COS_CASES["d768_f32_k100"]
    q, c, _ = cos_case_inputs(case)
    k = case["k"]
    s_full, r_full = R.cosine_topk(q, c, k)
    parts_s, parts_r = [], []
    bounds = np.linspace(0, c.shape[0], 9).astype(int)
    for a, b in zip(bounds[:-1], bounds[1:]):
        # shard-local normalisation is per row, so a shard's scores equal the full ones
        s, r = R.cosine_topk(q, c[a:b], k)
        parts_s.append(s)
        parts_r.append(np.where(r >= 0, r + a, -1))
    ms, mr = R.merge_topk(np.stack(parts_s), np.stack(parts_r), k)
    np.testing.assert_array_equal(mr, r_full)
    np.testing.assert_allclose(ms, s_full, atol=1e-15)


@pytest.mark.parametrize("name", sorted(COS_CASES))
@pytest.mark.parametrize("block", [1, 517, 4096])
def test_stream_oracle_matches_golden(name, block):
    """The block-streaming oracle (used at the BASELINE workload sizes) equals the golden
    sklearn + pandas vectors for any block size, exclusions included."""
    case = COS_CASES[name]
    gold = np.load(os.path.join(GOLD, "cos_topk_small.npz"))
    q, c, excl = cos_case_inputs(case)
    if block == 1:
        block = 257  # 1-row blocks take too long on CPU; 257 still splits every tile
    chunks = ((r0, c[r0:r0 + block]) for r0 in range(0, c.shape[0], block))
    s, r = R.cosine_topk_stream(q, chunks, case["k"], excl, workers=4)
    np.testing.assert_array_equal(r, gold[f"{name}_rows"])
    np.testing.assert_allclose(s, gold[f"{name}_scores"], rtol=0, atol=1e-12)


def test_stream_oracle_ties_across_blocks():
    """Equal scores split over blocks still come out (score desc, row asc)."""
    rng = np.random.default_rng(7)
    base = rng.standard_normal((5, 16))
    c = np.concatenate([base[rng.integers(0, 5, 300)], rng.standard_normal((100, 16))])
    q = base[:3] * 2.0
    s_ref, r_ref = R.cosine_topk(q, c, 40)
    for block in (7, 64, 400):
        chunks = ((r0, c[r0:r0 + block]) for r0 in range(0, c.shape[0], block))
        s, r = R.cosine_topk_stream(q, chunks, 40, workers=3)
        np.testing.assert_array_equal(r, r_ref)
        np.testing.assert_allclose(s, s_ref, rtol=0, atol=1e-15)
