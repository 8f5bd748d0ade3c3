"""Probe: can one batch's first pass (search.run_pipeline: query prep, sample, filter GEMM,
merges, rescore + certificate) be captured into a HIP graph and replayed, and what does a
replay save against eager launches at C2 (0.3-ms steps, ~7 kernels)? Measurement only; the
product path launches eagerly.

    python tools/graph_probe.py [--config C2] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import search  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    ebt.load()
    cat = ebt.Catalog(bench.make_catalog_shard(cfg, 0, cfg["n"], dev))
    q = bench.make_queries(cfg, dev)
    k = cfg["k"]
    kp = search.default_kprime(cat, k)

    def first_pass():
        qb = search.prepare_queries(cat, queries=q)
        return search.run_pipeline(cat, qb, k, kp, None, None, None)

    ref = first_pass()
    torch.cuda.synchronize()
    out = {"config": a.config}
    t0 = time.perf_counter()
    for _ in range(a.iters):
        first_pass()
    torch.cuda.synchronize()
    out["eager_ms"] = round((time.perf_counter() - t0) * 1e3 / a.iters, 4)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    try:
        with torch.cuda.stream(s):
            first_pass()               # warm-up on the capture stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            res = first_pass()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 -- report what refused capture
        out["capture"] = f"failed: {type(e).__name__}: {str(e)[:300]}"
        print(json.dumps(out), flush=True)
        return
    out["capture"] = "ok"
    g.replay()
    torch.cuda.synchronize()
    out["replay_equals_eager"] = bool(torch.equal(res[1], ref[1]) and
                                      torch.equal(res[0].nan_to_num(-9), ref[0].nan_to_num(-9)))
    t0 = time.perf_counter()
    for _ in range(a.iters):
        g.replay()
    torch.cuda.synchronize()
    out["graph_ms"] = round((time.perf_counter() - t0) * 1e3 / a.iters, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
