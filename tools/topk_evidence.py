"""HBM-bound kernels of the recommend path, timed on their launch stream (GPU).

    python tools/topk_evidence.py [--n 1000000] [--d 1536] [--b 4096] [--k 100]

For the C3 shape (1M x 1536 f32 catalog, 4096 queries, top-100):
  * row_norms_kernel   (catalog load: n*d*4 bytes read + n*12 written)
  * screen_image_kernel (catalog load: n*d*4 read + n*8 gnorm + n*d_pad*2 written)
  * select_topk_kernel (the unfused path's streaming select over a 4096 x n f32 score matrix:
                        B*n*4 bytes read + B*k'*12 written), k' = 200 as the pipeline uses
  * rescore_kernel     (exact float64 rescore of the screened list: the gathered catalog rows,
                        counted by replaying the kernel's two-stage cut in torch float64)
Each is run `iters` times back to back on torch's current stream (the one libebert launches
on), bracketed by torch.cuda.Event; prints one JSON object per kernel with GB/s and the fraction
of the 8 TB/s HBM peak. Run it under `rocprofv3 --kernel-trace --stats` for the per-kernel
average duration (profiles/r2_topk_kernel_stats.csv).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import _lib as L  # noqa: E402

PEAK = 8000.0


def timeit(fn, iters, warm=2):
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


def report(name, ms, nbytes, **kw):
    gbs = nbytes / (ms * 1e-3) / 1e9
    out = {"kernel": name, "ms": round(ms, 4), "bytes": int(nbytes), "GBps": round(gbs, 1),
           "frac_8000": round(gbs / PEAK, 4)}
    out.update(kw)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--skip-select", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ebt.load()
    st = L.stream_of(dev)
    n, d, B, k = args.n, args.d, args.b, args.k
    g = torch.Generator(device=dev).manual_seed(1)
    emb = torch.randn((n, d), generator=g, device=dev)
    cat = ebt.Catalog(emb)
    torch.cuda.synchronize()

    gn = torch.empty(n, dtype=torch.float64, device=dev)
    inv = torch.empty(n, dtype=torch.float32, device=dev)
    ms = timeit(lambda: L.call("ebt_row_norms", L.ptr(emb), L.EBT_F32, n, d, d, L.ptr(gn),
                               L.ptr(inv), st), args.iters)
    report("row_norms_kernel", ms, n * d * 4 + n * 12, shape=[n, d], dtype="f32")
    img = torch.empty((n, cat.ld_img), dtype=torch.float16, device=dev)
    ms = timeit(lambda: L.call("ebt_screen_image", L.ptr(emb), L.EBT_F32, n, d, d, L.ptr(cat.gnorm),
                               1, L.EBT_F16, L.ptr(img), cat.ld_img, st), args.iters)
    report("screen_image_kernel", ms, n * d * 4 + n * 8 + n * cat.ld_img * 2, shape=[n, d])
    del gn, inv, img

    kp = 200
    if not args.skip_select:
        # a Gaussian score matrix of the C3 magnitude (cosines ~ N(0, 1/d)), pitch as the pipeline's
        ld = (n + 63) // 64 * 64 + 64
        S = torch.randn((B, ld), generator=g, device=dev) * (d ** -0.5)
        ov = torch.empty((B, kp), device=dev)
        oi = torch.empty((B, kp), dtype=torch.int64, device=dev)
        for segs in (1, 2):
            if segs == 1:
                fn = lambda: L.call("ebt_select_topk", L.ptr(S), None, ld, B, n, 0, kp, 1,
                                    L.ptr(ov), L.ptr(oi), kp, st)
            else:
                sv = torch.empty((B, segs * kp), device=dev)
                si = torch.empty((B, segs * kp), dtype=torch.int64, device=dev)

                def fn():
                    L.call("ebt_select_topk", L.ptr(S), None, ld, B, n, 0, kp, segs, L.ptr(sv),
                           L.ptr(si), segs * kp, st)
                    L.call("ebt_select_topk", L.ptr(sv), L.ptr(si), segs * kp, B, segs * kp, 0,
                           kp, 1, L.ptr(ov), L.ptr(oi), kp, st)
            ms = timeit(fn, args.iters)
            report("select_topk_kernel", ms, B * n * 4 + B * kp * 12, shape=[B, n], kprime=kp,
                   segs=segs)
        # correctness spot check of the select against torch.topk on 4 rows
        L.call("ebt_select_topk", L.ptr(S), None, ld, B, n, 0, kp, 1, L.ptr(ov), L.ptr(oi), kp, st)
        ref = torch.topk(S[:4, :n], kp, dim=1)
        print(json.dumps({"select_check_rows_equal": bool(torch.equal(
            torch.sort(ref.indices, 1)[0], torch.sort(oi[:4], 1)[0]))}), flush=True)
        del S

    # rescore: the screened list of a C3 batch, then the kernel alone
    q = torch.randn((B, d), generator=g, device=dev)
    qb = ebt.search.prepare_queries(cat, queries=q)
    lv, lr, ovf, eps = ebt.search.run_screen(cat, qb, k, kp)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    cert = torch.empty(B, dtype=torch.int32, device=dev)

    def rs():
        L.call("ebt_rescore", L.ptr(qb.q64), B, d, L.ptr(emb), L.EBT_F32, d, L.ptr(cat.gnorm), 0,
               L.ptr(lv), L.ptr(lr), kp, k, n, L.ptr(eps), None, L.ptr(out_s), L.ptr(out_r),
               L.ptr(cert), None, st)
    ms = timeit(rs, args.iters)
    # replay the two-stage cut: pass A gathers the list's first k rows; pass B the rest with
    # approx >= max(approx[k-1] - 2 eps, s_min - eps)
    e64 = eps[:B].double()[:, None]
    cut = lv[:, k - 1:k].double() - 2 * e64
    valid = lr >= 0
    rows = lr.clamp(min=0)
    top_exact = (qb.q64[:, None, :] * emb[rows[:, :k]].double()).sum(-1) / cat.gnorm[rows[:, :k]]
    smin = top_exact.min(1, keepdim=True).values
    cut2 = torch.maximum(cut, smin - e64)
    rest = valid[:, k:] & (lv[:, k:].double() >= cut2)
    gathered = int(valid[:, :k].sum()) + int(rest.sum())
    nbytes = gathered * (d * 4 + 8) + B * kp * 12 + B * d * 8 + B * k * 16
    report("rescore_kernel", ms, nbytes, rows_gathered_per_query=round(gathered / B, 1),
           kprime=kp, certified=int((cert == 1).sum()))


if __name__ == "__main__":
    main()
