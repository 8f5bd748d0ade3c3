"""The float64 paths outside the fused screen, timed: the large-k path (min(k, n) > 4096: every
score in float64, sorted) and the exact fallback screen (EBT_FLAG_EXACT).

    python tools/exact_bench.py [--n 200000] [--d 768] [--b 64]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import _lib, search  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--b", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    cat = ebt.Catalog(torch.randn((a.n, a.d), generator=g, device=dev))
    q = torch.randn((a.b, a.d), generator=g, device=dev)
    out = {"lib": os.environ.get("EBERT_LIB", "default"), "n": a.n, "d": a.d, "b": a.b}
    qb = search.prepare_queries(cat, queries=q)
    kp = search.default_kprime(cat, 100)
    for name, fn in (("large_k_5000", lambda: ebt.score_topk(cat, 5000, queries=q)),
                     ("exact_screen_k100", lambda: search.run_pipeline(
                         cat, qb, 100, kp, flags=_lib.EBT_FLAG_EXACT))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out[name + "_ms"] = round((time.perf_counter() - t0) * 1e3 / 3, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
