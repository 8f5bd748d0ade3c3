"""Filter-GEMM cost per fused-screen segment (GPU): for the bench's segment schedule, the filter
kernel over s rows with the threshold the pilot/segment scheme would have (k'-th of the r rows
seen so far, Gaussian quantile), vs the same launch with no hits (threshold +inf).

    python tools/seg_bench.py [--n 1000000] [--b 4096] [--d 1536] [--kprime 200]
"""
import argparse
import json
import os
import sys

import torch
from scipy.stats import norm

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robot_ebert_amd import _lib as L  # noqa: E402
from kernel_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--kprime", type=int, default=200)
    ap.add_argument("--segs", default=None, help="r:s,... (default: 3x growth from 1024, cap 524288)")
    ap.add_argument("--no-inf", action="store_true", help="skip the no-hit comparison launch")
    ap.add_argument("--hits", default=None, help="h1,h2,...: one launch over --n rows per target "
                    "hits/query (Gaussian quantile threshold)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    L.load()
    B, d = a.b, a.d
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn((B, d), generator=g, device=dev).half()
    c = torch.randn((a.n, d), generator=g, device=dev).half()
    qs = torch.ones(B, device=dev)
    st = L.stream_of(dev)
    G = L.load().ebt_filter_group_rows(B)
    if a.hits:
        segs = [(max(1, round(a.kprime * a.n / float(h))), a.n) if float(h) > 0 else (10**12, a.n)
                for h in a.hits.split(",")]
    elif a.segs:
        segs = [tuple(int(x) for x in t.split(":")) for t in a.segs.split(",")]
    else:
        segs, r = [], 1024
        while r < a.n:
            s = min(3 * r, 524288, a.n - r)
            segs.append((r, s))
            r += s
    total_ms = total_ms0 = 0.0
    for (r, s) in segs:
        groups = (s + G - 1) // G
        p = min(0.5, a.kprime / r)
        thr = torch.full((B,), float(norm.isf(p)) * d ** 0.5, device=dev)
        exp_hits = p * s
        slots = max(16, min(128, int(4 * exp_hits / groups + 8 + 15) // 16 * 16))
        cand = torch.empty((B, groups * slots), dtype=torch.int64, device=dev)
        counts = torch.empty((B, groups), dtype=torch.uint8, device=dev)
        ovf = torch.zeros(B, dtype=torch.int32, device=dev)
        cv = c[r:r + s] if r + s <= a.n else c[:s]

        def run(t):
            L.call("ebt_screen_filter", L.ptr(q), B, L.ptr(cv), s, d, d, L.DTYPE_CODE[torch.float16],
                   L.ptr(qs), None, L.ptr(t), L.ptr(cand), groups * slots, slots, L.ptr(counts),
                   groups, L.ptr(ovf), 0, st)
        ms = timeit(lambda: run(thr))
        hits = float(counts.float().sum(1).mean())
        inf = torch.full_like(thr, float("inf"))
        ms0 = timeit(lambda: run(inf)) if not a.no_inf else float("nan")
        total_ms += ms
        total_ms0 += ms0
        tf = 2.0 * B * s * d / (ms * 1e-3) / 1e12
        tf0 = 2.0 * B * s * d / (ms0 * 1e-3) / 1e12
        print(json.dumps({"r": r, "s": s, "slots": slots, "hits": round(hits, 1),
                          "ms": round(ms, 4), "tflops": round(tf, 1), "ms_nohit": round(ms0, 4),
                          "tflops_nohit": round(tf0, 1)}), flush=True)
    print(json.dumps({"total_ms": round(total_ms, 3), "total_ms_nohit": round(total_ms0, 3)}))


if __name__ == "__main__":
    main()
