"""Per-kernel microbenchmarks (GPU): screening GEMM TFLOP/s and streaming select GB/s.

    python tools/kernel_bench.py [--gemm] [--select] [--rescore]

Timed with torch.cuda.Event on the current stream, which is the stream libebert launches on.
Random (Gaussian) operands: zero-filled data runs faster on this chip (DVFS), see the guide.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robot_ebert_amd import _lib as L  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def bench_gemm(dev, B, N, d, dt):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn((B, d), generator=g, device=dev).to(dt)
    c = torch.randn((N, d), generator=g, device=dev).to(dt)
    qs = torch.ones(B, device=dev)
    S = torch.empty((B, N), device=dev)
    st = L.stream_of(dev)
    code = L.DTYPE_CODE[dt]
    ms = timeit(lambda: L.call("ebt_screen_scores", L.ptr(q), B, L.ptr(c), N, d, d, code,
                               L.ptr(qs), None, L.ptr(S), N, st))
    tf = 2.0 * B * N * d / (ms * 1e-3) / 1e12
    # fused-screen (filter) epilogue: threshold high enough that ~0.3% of scores are kept
    thr = torch.full((B,), 0.0, device=dev)
    thr[:] = 3.0 * (d ** 0.5)  # raw (unnormalised) Gaussian dot products: ~3 sigma
    if os.environ.get("EBT_KB_THR") == "inf":  # no hits at all (ablation runs)
        thr[:] = float("inf")
    G = L.load().ebt_filter_group_rows(B)
    groups = (N + G - 1) // G
    slots = 16
    cand = torch.empty((B, groups * slots), dtype=torch.int64, device=dev)
    counts = torch.empty((B, groups), dtype=torch.uint8, device=dev)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)

    def run_filter():
        L.call("ebt_screen_filter", L.ptr(q), B, L.ptr(c), N, d, d, code, L.ptr(qs), None,
               L.ptr(thr), L.ptr(cand), groups * slots, slots, L.ptr(counts), groups,
               L.ptr(ovf), 0, st)
    ms_f = timeit(run_filter)
    tf_f = 2.0 * B * N * d / (ms_f * 1e-3) / 1e12
    return {"kernel": "screen_gemm", "B": B, "N": N, "d": d, "dtype": str(dt), "ms": round(ms, 4),
            "tflops": round(tf, 1), "frac_2500": round(tf / 2500, 4),
            "filter_ms": round(ms_f, 4), "filter_tflops": round(tf_f, 1),
            "mean_hits": round(float(counts.float().sum(1).mean()), 1),
            "overflow": int(ovf.sum())}


def bench_select(dev, B, n, kp):
    g = torch.Generator(device=dev).manual_seed(0)
    v = torch.randn((B, n), generator=g, device=dev) * 0.0255
    ov = torch.empty((B, kp), device=dev)
    oi = torch.empty((B, kp), dtype=torch.int64, device=dev)
    st = L.stream_of(dev)
    ms = timeit(lambda: L.call("ebt_select_topk", L.ptr(v), None, n, B, n, 0, kp, 1, L.ptr(ov),
                               L.ptr(oi), kp, st))
    gbs = 4.0 * B * n / (ms * 1e-3) / 1e9
    return {"kernel": "select_topk", "B": B, "n": n, "kprime": kp, "ms": round(ms, 4),
            "GBps": round(gbs, 1), "frac_8000": round(gbs / 8000, 4)}


def bench_merge(dev, B, kp, groups, hits, slots=16):
    """ebt_merge_hits: a sorted k' list per query + `hits` hits spread over `groups` groups."""
    g = torch.Generator(device=dev).manual_seed(0)
    fv = torch.sort(torch.rand((B, kp), generator=g, device=dev), dim=1, descending=True)[0]
    fi = torch.arange(kp, device=dev).repeat(B, 1) + 10_000_000
    grp = torch.randint(0, groups, (B, hits), generator=g, device=dev)
    counts = torch.zeros((B, (groups + 15) // 16 * 16), dtype=torch.uint8, device=dev)
    ones = torch.ones_like(grp, dtype=torch.uint8)
    counts.scatter_add_(1, grp, ones)
    counts.clamp_(max=slots)
    cand = torch.zeros((B, groups * slots), dtype=torch.int64, device=dev)
    # composite: key of a score in [0,1) << 32 | ~row
    key = (torch.rand((B, groups * slots), generator=g, device=dev) * 2**30).long() + 2**31
    row = torch.arange(groups * slots, device=dev).repeat(B, 1)
    cand[:] = (key << 32) | ((~row) & 0xFFFFFFFF)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    st = L.stream_of(dev)
    fv0, fi0 = fv.clone(), fi.clone()

    def run():
        fv.copy_(fv0)
        fi.copy_(fi0)
        L.call("ebt_merge_hits", L.ptr(fv), L.ptr(fi), B, kp, min(100, kp), L.ptr(cand), groups * slots, slots,
               L.ptr(counts), counts.shape[1], groups, 0, None, None, L.ptr(ovf), st)
    ms = timeit(run)
    ms_copy = timeit(lambda: (fv.copy_(fv0), fi.copy_(fi0)))
    return {"kernel": "merge_hits", "B": B, "kprime": kp, "groups": groups, "hits": hits,
            "ms": round(ms - ms_copy, 4), "ovf": int(ovf.sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", action="store_true")
    ap.add_argument("--select", action="store_true")
    ap.add_argument("--merge", action="store_true")
    ap.add_argument("--merge-shape", default=None, help="B,kprime,groups,hits for --merge")
    ap.add_argument("--one", action="store_true", help="single C3-chunk GEMM config (profiling)")
    ap.add_argument("--shape", default="4096,262144,1536", help="B,N,d for --one")
    ap.add_argument("--select-shapes", default=None,
                    help="B,n,kprime;... for --select (default: the pipeline's shapes)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    L.load()
    res = []
    if args.merge:
        cfgs = [(4096, 200, 2048, 400), (4096, 200, 48, 400), (4096, 200, 2048, 50),
                (4096, 200, 2048, 800), (4096, 1016, 2048, 1000)]
        if args.merge_shape:
            cfgs = [tuple(int(x) for x in args.merge_shape.split(","))]
        for (B, kp, groups, hits) in cfgs:
            print(json.dumps(bench_merge(dev, B, kp, groups, hits)), flush=True)
        return
    if args.one:
        B, N, d = (int(x) for x in args.shape.split(","))
        print(json.dumps(bench_gemm(dev, B, N, d, torch.float16)), flush=True)
        return
    if args.gemm or not args.select:
        for (B, N, d, dt) in [(4096, 262144, 1536, torch.float16), (4096, 262144, 1536, torch.bfloat16),
                              (1024, 100000, 768, torch.bfloat16), (4096, 65536, 1536, torch.float16)]:
            res.append(bench_gemm(dev, B, N, d, dt))
            print(json.dumps(res[-1]), flush=True)
    if args.select or not args.gemm:
        shapes = [(4096, 262144, 200), (4096, 262144, 104), (1024, 100000, 120)]
        if args.select_shapes:
            shapes = [tuple(int(x) for x in t.split(",")) for t in args.select_shapes.split(";")]
        for (B, n, kp) in shapes:
            res.append(bench_select(dev, B, n, kp))
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
