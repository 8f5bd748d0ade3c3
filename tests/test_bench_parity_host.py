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
