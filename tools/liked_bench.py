"""Query prep for liked-movie users (lib.py:52: the mean of the liked rows' cosine rows, folded
into one query per user) at the C3 catalog: B users with L liked rows each, hipEvent-timed,
against the dense-query prep of the same batch.

    python tools/liked_bench.py [--b 4096] [--liked 20] [--iters 20]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import search  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--liked", type=int, default=20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--unaligned", action="store_true",
                    help="catalog rows at stride d + 1 (the element form of ebt_query_liked_sum)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    ebt.load()
    emb = bench.make_catalog_shard(cfg, 0, cfg["n"], dev)
    if a.unaligned:
        wide = torch.empty((cfg["n"], cfg["d"] + 1), dtype=emb.dtype, device=dev)
        wide[:, :cfg["d"]] = emb
        emb = wide[:, :cfg["d"]]
    cat = ebt.Catalog(emb)
    rng = np.random.default_rng(0)
    liked = [sorted(rng.choice(cfg["n"], a.liked, replace=False).tolist()) for _ in range(a.b)]
    lk = search.csr_from_lists(liked, dev)
    q = bench.make_queries(cfg, dev)[:a.b].contiguous()
    ms_liked = timed(lambda: search.prepare_queries(cat, liked=lk), a.iters)
    ms_dense = timed(lambda: search.prepare_queries(cat, queries=q), a.iters)
    rows_read = a.b * a.liked
    print(json.dumps({"config": a.config, "users": a.b, "liked_per_user": a.liked,
                      "form": "element (ld = d + 1)" if a.unaligned else "vector",
                      "liked_prep_ms": round(ms_liked, 4), "dense_prep_ms": round(ms_dense, 4),
                      "liked_rows_GBps": round(rows_read * cfg["d"] * 4 / ms_liked / 1e6, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
