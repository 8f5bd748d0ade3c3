"""CPU: bench.py's N > 1 parity plumbing (global_blocks + oracle_parity).

At N > 1 rank 0 holds only its shard, so bench.py regenerates the WHOLE catalog block by block
from the seeds every shard was made from and streams it into the host oracle. Here the same
functions run on the CPU on a small catalog that spans several 65536-row seed blocks: the
regenerated blocks equal the catalog built in one piece, a result equal to the oracle's passes,
and a result with two rows swapped or a row replaced fails.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import restatement as R  # noqa: E402

CFG = dict(n=140_000, d=8, dtype="f32", b=6, k=5)


def _whole():
    return bench.make_catalog_shard(CFG, 0, CFG["n"], torch.device("cpu"))


def test_global_blocks_equal_the_catalog():
    cat = _whole().numpy()
    got = np.concatenate([b for _, b in bench.global_blocks(CFG, torch.device("cpu"),
                                                            block=50_000)])
    assert got.shape == cat.shape and np.array_equal(got, cat)
    # a shard generated alone holds the same rows as that slice of the whole
    shard = bench.make_catalog_shard(CFG, 70_000, 140_000, torch.device("cpu")).numpy()
    assert np.array_equal(shard, cat[70_000:])


def test_oracle_parity_accepts_exact_and_rejects_wrong():
    cat = _whole().numpy().astype(np.float64)
    q = np.random.default_rng(5).standard_normal((CFG["b"], CFG["d"]))
    s, r = R.cosine_topk(q, cat, CFG["k"])
    blocks = lambda: bench.global_blocks(CFG, torch.device("cpu"), block=50_000)  # noqa: E731
    ok = bench.oracle_parity(CFG["k"], blocks(), q, torch.from_numpy(s), torch.from_numpy(r),
                             CFG["b"], "test")
    assert ok["rows_bit_exact"] and ok["max_abs_score_diff"] <= 1e-12
    assert ok["queries_checked"] == CFG["b"]
    r_swap = r.copy()
    r_swap[0, [0, 1]] = r_swap[0, [1, 0]]
    bad = bench.oracle_parity(CFG["k"], blocks(), q, torch.from_numpy(s),
                              torch.from_numpy(r_swap), CFG["b"], "test")
    assert not bad["rows_bit_exact"]
    r_repl = r.copy()
    r_repl[3, 4] = (r_repl[3, 4] + 1) % CFG["n"]
    bad = bench.oracle_parity(CFG["k"], blocks(), q, torch.from_numpy(s),
                              torch.from_numpy(r_repl), CFG["b"], "test")
    assert not bad["rows_bit_exact"]


def test_cpu_baseline_over_regenerated_global_catalog():
    """N > 1: rank 0's cpu_baseline + parity run over the WHOLE catalog regenerated from its
    seeds (global_blocks), not over its shard: the (i)/(ii) keys are there and the parity of the
    oracle's own answer passes."""
    cat = _whole().numpy().astype(np.float64)
    q = torch.from_numpy(np.random.default_rng(6).standard_normal((CFG["b"], CFG["d"])))
    s, r = R.cosine_topk(q.numpy(), cat, CFG["k"])
    base, par = bench.cpu_baseline_and_parity(
        CFG, lambda rows: bench.global_blocks(CFG, torch.device("cpu"), block=50_000, rows=rows),
        CFG["n"], q, torch.from_numpy(s), torch.from_numpy(r), budget_s=0.2, n_parity=CFG["b"],
        what="whole global catalog")
    for key in ("value", "unit", "cores", "kind", "sample", "batched", "host"):
        assert key in base, key
    assert base["value"] > 0 and base["batched"]["value"] > 0 and base["kind"] == "port"
    assert par["rows_bit_exact"] and par["queries_checked"] == CFG["b"]
    assert par["oracle"].endswith("whole global catalog")


def test_traffic_reason_and_stage_breakdown():
    """The N > 1 line's roofline.traffic is null WITH a reason when no PMC summary exists for
    that config/N; the stage breakdown sums the recorded stages and reports the rest."""
    v, why = bench.pmc_traffic("C3", 8)
    assert v is None and "PMC" in why
    v1, note = bench.pmc_traffic("C3", 1)
    assert v1 is not None and v1 > 0 and note.startswith("profiles/pmc_C3_n1.json")
    st = {"gemm_filter": (1.0, 3), "rescore": (0.25, 1), "collective_wait": (0.05, 3)}
    b = bench.stage_breakdown(st, 1.5, 8)
    assert b["sum_ms"] == 1.3 and abs(b["rest_ms"] - 0.2) < 1e-9
    from robot_ebert_amd._lib import STAGES
    for name in ("rescore", "shard_merge", "collective_wait", "prep", "small"):
        assert name in STAGES


def test_exclusion_variant_parity():
    """bench.py --exclude R: seeded per-query exclusions (sorted, distinct, in range); the parity
    sample drops them in the oracle as lib.py:55 does, accepts an answer without them and counts
    an excluded row that comes back."""
    ex = bench.make_exclusions(CFG, 40)
    assert len(ex) == CFG["b"]
    for e in ex:
        assert 0 < len(e) <= 40 and np.all(np.diff(e) > 0) and e[0] >= 0 and e[-1] < CFG["n"]
    assert all(np.array_equal(a, b) for a, b in zip(ex, bench.make_exclusions(CFG, 40)))
    cat = _whole().numpy().astype(np.float64)
    q = np.random.default_rng(7).standard_normal((CFG["b"], CFG["d"]))
    # the plain top-k's first row of query 0 excluded: the exclusion changes the answer
    s0, r0 = R.cosine_topk(q, cat, CFG["k"])
    ex[0] = np.union1d(ex[0], r0[0, :1])
    s, r = R.cosine_topk(q, cat, CFG["k"], [e.tolist() for e in ex])
    assert r[0, 0] != r0[0, 0]
    blocks = lambda: bench.global_blocks(CFG, torch.device("cpu"), block=50_000)  # noqa: E731
    ok = bench.oracle_parity(CFG["k"], blocks(), q, torch.from_numpy(s), torch.from_numpy(r),
                             CFG["b"], "test", exclude=ex)
    assert ok["rows_bit_exact"] and ok["excluded_rows_returned"] == 0
    bad = bench.oracle_parity(CFG["k"], blocks(), q, torch.from_numpy(s0),
                              torch.from_numpy(r0), CFG["b"], "test", exclude=ex)
    assert not bad["rows_bit_exact"] and bad["excluded_rows_returned"] >= 1


def test_line_dtype_is_the_result_arithmetic():
    """the line's `dtype` names the arithmetic of the returned scores (float64,
    the reference's own: constants.py:56, lib.py:51), not the screen's operand type, which
    config.arith / config.screen_operands carry."""
    for name, ops in (("C2", "bf16"), ("C3", "f16"), ("C4", "bf16"), ("C5", "f16")):
        lab = bench.arith_labels(bench.CONFIGS[name])
        assert lab["dtype"] == "f64"
        assert lab["screen_operands"] == ops
        assert "f64" in lab["arith"] and ops in lab["arith"] and "certified" in lab["arith"]
