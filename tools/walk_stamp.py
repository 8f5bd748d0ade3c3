"""The persistent screening GEMM's tile walk, measured (why C4 / C5 launches
fetch 2.6x what the a x b window model predicts).

    python tools/walk_stamp.py [--n 520192] [--b 16384] [--d 1536] [--img f16] [--cscale]

Loads the diagnostic build _abl/libebert_walk.so (tools/abl_build.sh walk -DEBT_WALK_STAMP):
lane 0 of every workgroup of a filter-mode launch records (tile index L, 100 MHz real time) at
the start of each of its tiles and at exit. After warm-up launches of one filter segment (B
queries x n rows x d, a threshold at --z sigmas of the cosine), one stamped launch gives, per XCD
(workgroup b runs on XCD b % 8):
  * the window in flight: at 400 instants, the tile indices the XCD's workgroups are working on;
    spread = max - min + 1 (a lockstep walk keeps it at the XCD's workgroup count, 32), and the
    distinct catalog / query tiles among them;
  * the drift: per workgroup, the finish time of its t-th tile minus the XCD's median at t;
  * an L2 model: each tile's K-loop touches its catalog and query tile's 32 KiB K-slices in
    order over its measured duration; a 4 MiB LRU per XCD over those slices, fed the measured
    schedule, gives the L2 miss bytes -- next to the same LRU fed the ideal lockstep schedule
    (every workgroup's t-th tile over the same time span), i.e. what the drift costs in fetch.
One JSON line per launch shape. Compare fetch_model_gb with rocprofv3 --pmc FETCH_SIZE of the
same command (x 2 KiB on gfx950).
"""
import argparse
import collections
import ctypes
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VP, I32, I64, INT = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int
WALK_MAX = 4096
SLICE = 256 * 64 * 2          # one 256-row x 64-k f16 K-slice of a tile
L2_BYTES = 4 << 20


def lru_misses(events, cap):
    """events: iterable of keys in time order; misses of an LRU of `cap` keys."""
    lru = collections.OrderedDict()
    miss = 0
    for key in events:
        if key in lru:
            lru.move_to_end(key)
        else:
            miss += 1
            lru[key] = None
            if len(lru) > cap:
                lru.popitem(last=False)
    return miss


def xcd_events(tiles, n_qt, ktiles, lockstep):
    """tiles: list of (L, t_start, t_end) of one XCD's workgroups (all of them). Returns the
    K-slice keys ('c', ct, k) / ('q', qt, k) in time order: K-step k of a tile at
    t_start + (k + 0.5) / ktiles x 0.9 x duration (the last 10 % is its epilogue)."""
    ev = []
    for (L, t0, t1) in tiles:
        g, w = divmod(L, 4 * n_qt)
        # the walk's group of 4 catalog tiles walked query-tile-major (full groups)
        ct, qt = g * 4 + (w & 3), w >> 2
        for k in range(ktiles):
            t = t0 + (k + 0.5) / ktiles * 0.9 * (t1 - t0)
            ev.append((t, 0, ct, k))
            ev.append((t, 1, qt, k))
    ev.sort()
    return [(e[1], e[2], e[3]) for e in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=520_192)
    ap.add_argument("--b", type=int, default=16384)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--z", type=float, default=3.0)
    ap.add_argument("--img", default="f16", choices=["f16", "bf16"])
    ap.add_argument("--cscale", action="store_true")
    ap.add_argument("--warm", type=int, default=6)
    ap.add_argument("--lib", default=os.path.join(ROOT, "_abl", "libebert_walk.so"))
    ap.add_argument("--alloc-rows", type=int, default=0,
                    help="allocate this many catalog rows and screen the --n rows at --offset-rows "
                         "of it (the bench's C5 parts are 520K-row windows of a 50M-row catalog)")
    ap.add_argument("--offset-rows", type=int, default=0)
    ap.add_argument("--advance", action="store_true",
                    help="each warm-up launch screens the next --n rows of the allocation "
                         "(consecutive windows, as the bench's split parts) instead of the same")
    a = ap.parse_args()
    lib = ctypes.CDLL(a.lib)
    f = lib.ebt_screen_filter
    f.argtypes = [VP, I64, VP, I64, I32, I32, INT, VP, VP, VP, VP, I64, I32, VP, I64, VP, I64, VP]
    f.restype = INT
    lib.ebt_debug_walk_stamps.argtypes = [VP]
    lib.ebt_debug_walk_stamps.restype = INT
    lib.ebt_last_error.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    B, N, d = a.b, a.n, a.d
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn((B, d), generator=g, device=dev)
    q = (q / q.norm(dim=1, keepdim=True)).to(torch.float16 if a.img == "f16" else torch.bfloat16)
    if a.alloc_rows > N:
        big = torch.empty((a.alloc_rows, d), dtype=q.dtype, device=dev)
        for r0 in range(0, a.alloc_rows, 1 << 20):   # filled in 1M-row blocks (bounded temp)
            r1 = min(a.alloc_rows, r0 + (1 << 20))
            x = torch.randn((r1 - r0, d), generator=g, device=dev)
            big[r0:r1] = (x / x.norm(dim=1, keepdim=True)).to(q.dtype)
            del x
        c = big[a.offset_rows:a.offset_rows + N]
        windows = [big[a.offset_rows + i * N:a.offset_rows + (i + 1) * N]
                   for i in range(max(1, (a.alloc_rows - a.offset_rows) // N))]
    else:
        c = torch.randn((N, d), generator=g, device=dev)
        c = (c / c.norm(dim=1, keepdim=True)).to(q.dtype)
        windows = [c]
    idt = 2 if a.img == "f16" else 1
    qs = torch.ones(B, device=dev)
    cs = torch.ones(N, device=dev) if a.cscale else None
    G, slots = 256, 16
    groups = (N + G - 1) // G
    cand = torch.empty((B, groups * slots), dtype=torch.int64, device=dev)
    counts = torch.empty((B, groups), dtype=torch.uint8, device=dev)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    thr = torch.full((B,), a.z / d ** 0.5, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def launch(cc=None):
        cc = c if cc is None else cc
        rc = f(P(q), B, P(cc), N, d, d, idt, P(qs), P(cs) if cs is not None else None, P(thr),
               P(cand), groups * slots, slots, P(counts), groups, P(ovf), 0, st)
        if rc:
            raise RuntimeError(lib.ebt_last_error().decode())
    lib.ebt_debug_walk_stamps(None)
    for i in range(a.warm):
        launch(windows[i % len(windows)] if a.advance else None)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    launch()
    e.record()
    torch.cuda.synchronize()
    ms_plain = s.elapsed_time(e)
    stamps = torch.zeros(256 * WALK_MAX * 2, dtype=torch.int64, device=dev)
    lib.ebt_debug_walk_stamps(P(stamps))
    s.record()
    launch()
    e.record()
    torch.cuda.synchronize()
    lib.ebt_debug_walk_stamps(None)
    ms_stamped = s.elapsed_time(e)
    v = stamps.view(256, WALK_MAX, 2).cpu().numpy()
    n_qt, n_ct, ktiles = B // 256, (N + 255) // 256, d // 64
    per_xcd = collections.defaultdict(list)
    wg_tiles = {}
    for bid in range(256):
        rows = v[bid]
        last = np.nonzero(rows[:, 0] == -1)[0]
        if len(last) == 0:
            continue
        m = int(last[0])
        Ls, ts = rows[:m, 0].astype(np.int64), rows[:m + 1, 1].astype(np.float64) / 100.0  # us
        wg_tiles[bid] = [(int(Ls[i]), ts[i], ts[i + 1]) for i in range(m)]
        per_xcd[bid & 7].append(bid)
    t_all0 = min(t[0][1] for t in wg_tiles.values())
    t_all1 = max(t[-1][2] for t in wg_tiles.values())
    out = {"shape": [B, N, d], "img": a.img, "row_scales": bool(a.cscale), "query_tiles": n_qt,
           "alloc_rows": a.alloc_rows or N, "offset_rows": a.offset_rows,
           "catalog_tiles": n_ct, "tiles": n_qt * n_ct, "launch_ms": round(ms_plain, 3),
           "launch_ms_stamped": round(ms_stamped, 3),
           "tiles_per_workgroup": round(n_qt * n_ct / max(len(wg_tiles), 1), 1)}
    spreads, cts, qts, drift, miss_meas, miss_lock = [], [], [], [], 0, 0
    inst = np.linspace(t_all0, t_all1, 402)[1:-1]
    for x, bids in sorted(per_xcd.items()):
        tl = [wg_tiles[b] for b in bids]
        cols = []   # per workgroup: the tile index in progress at every instant (-1: none)
        for tiles in tl:
            L = np.array([x[0] for x in tiles])
            t0 = np.array([x[1] for x in tiles])
            t1 = np.array([x[2] for x in tiles])
            i = np.searchsorted(t0, inst, side="right") - 1
            ok = (i >= 0) & (inst < t1[np.clip(i, 0, None)])
            cols.append(np.where(ok, L[np.clip(i, 0, None)], -1))
        cols = np.stack(cols, 1)
        for row in cols:
            cur = [int(x) for x in row if x >= 0]
            if len(cur) >= 2:
                spreads.append(max(cur) - min(cur) + 1)
                cts.append(len({(L // (4 * n_qt)) * 4 + ((L % (4 * n_qt)) & 3) for L in cur}))
                qts.append(len({(L % (4 * n_qt)) >> 2 for L in cur}))
        depth = min(len(tiles) for tiles in tl)
        for i in range(depth):
            ends = np.array([tiles[i][2] for tiles in tl])
            drift.extend((ends - np.median(ends)).tolist())
        # L2 model: the measured schedule vs lockstep (the t-th tile of every workgroup over one
        # common span: the XCD's median start / end of its t-th tile)
        meas = [tt for tiles in tl for tt in tiles]
        miss_meas += lru_misses(xcd_events(meas, n_qt, ktiles, False), L2_BYTES // SLICE)
        lock = []
        for i in range(max(len(tiles) for tiles in tl)):
            have = [tiles[i] for tiles in tl if i < len(tiles)]
            t0 = float(np.median([h[1] for h in have]))
            t1 = float(np.median([h[2] for h in have]))
            lock.extend((h[0], t0, t1) for h in have)
        miss_lock += lru_misses(xcd_events(lock, n_qt, ktiles, True), L2_BYTES // SLICE)
    sp = np.asarray(spreads)
    dr = np.abs(np.asarray(drift))
    med_tile_us = float(np.median([t1 - t0 for tiles in wg_tiles.values() for (_, t0, t1) in tiles]))
    out.update({
        "window_spread_tiles": {"median": float(np.median(sp)), "p90": float(np.percentile(sp, 90)),
                                "lockstep": len(per_xcd[0])},
        "distinct_catalog_tiles_in_flight_median": float(np.median(cts)),
        "distinct_query_tiles_in_flight_median": float(np.median(qts)),
        "tile_us_median": round(med_tile_us, 2),
        "drift_us": {"median_abs": round(float(np.median(dr)), 2),
                     "p90_abs": round(float(np.percentile(dr, 90)), 2),
                     "max_abs": round(float(dr.max()), 2)},
        "drift_tiles_p90": round(float(np.percentile(dr, 90)) / med_tile_us, 2),
        "fetch_model_gb": round(miss_meas * SLICE / 1e9, 3),
        "fetch_model_lockstep_gb": round(miss_lock * SLICE / 1e9, 3),
        "operand_bytes_gb": round((N + B) * d * 2 / 1e9, 3),
        "model": "4 MiB LRU per XCD over 32 KiB K-slices, K-steps spread over 90 % of each "
                 "tile's measured duration"})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
