"""First-pass certificate histogram of one bench configuration (EBERT_LIB picks the library):
how many queries the retries of ebt_cosine_topk_finish rerun, and what they cost.
    EBERT_LIB=... python tools/cert_ab.py --config C5 --n 6250000"""
import argparse
import collections
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from robot_ebert_amd import Catalog  # noqa: E402
from robot_ebert_amd import search  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--n", type=int, default=0)
    a = ap.parse_args()
    cfg = dict(bench.CONFIGS[a.config])
    if a.n:
        cfg["n"] = a.n
    dev = torch.device("cuda:0")
    emb = bench.make_catalog_shard(cfg, 0, cfg["n"], dev)
    cat = Catalog(emb)
    q = bench.make_queries(cfg, dev)
    out = {"lib": os.environ.get("EBERT_LIB", "tree"), "config": a.config, "n": cfg["n"]}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = search.score_topk_submit(cat, cfg["k"], queries=q)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        hist = collections.Counter(int(x) for x in p.cert_host[:cfg["b"]].tolist())
        search.score_topk_finish(p)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"rep{rep}"] = {"first_pass_ms": round(1e3 * (t1 - t0), 2),
                            "finish_ms": round(1e3 * (t2 - t1), 2),
                            "cert_hist": {str(k): v for k, v in sorted(hist.items())}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
