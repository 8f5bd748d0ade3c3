"""C5 on 8 ranks at its REAL shard size, on one MI355X ("the C5 8-shard
protocol at its real 6.25M-row shard size has never executed").

BASELINE's C5 (50M x 1536 f16, 16384 queries, top-1000) row-sharded over 8 ranks: eight
6.25M-row shards (19.2 GB each, 153.6 GB together) and eight ranks' sharded workspaces (one slot
each: ebt_sharded_workspace_bytes, 11.5 GiB with the comm's all-reduce slot set -- the dense
path never calls it) fit one 288 GB GPU only since round 6 trimmed the speculative screen's
layout (27.8 GiB per slot before). The ranks run as threads through the C ABI's step
(distributed.ShardedTopk -> ebt_cosine_topk_sharded_submit / _finish / _wait), every all-gather
a barrier exchange between the threads, ONE batch. Checked: every rank returns the same merged
global top-1000; the merged rows of `--sample` queries equal the host float64 oracle over all
50M rows (oracle/restatement.py, streamed from the shards); properties of every query (sorted,
distinct, in range). Prints one JSON line.

    python tools/c5_full_shards.py [--sample 16]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402
from oracle import restatement as R  # noqa: E402  (the checker only)
from robot_ebert_amd import _lib  # noqa: E402
from robot_ebert_amd.distributed import ShardedTopk, TorchGatherComm, shard_range  # noqa: E402


def log(m):
    print(m, file=sys.stderr, flush=True)


class _AllReduceSlot(TorchGatherComm):
    """TorchGatherComm with the comm's optional all_reduce_f64 set to a callback that is never
    called on the dense path: the workspace then has no room for the liked path's gathered
    partial sums (R x B x d x 8 bytes = 1.5 GiB per rank at C5)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)

        def never(ctx, buf, count, stream):
            return -1
        self._ar = _lib.ALLREDUCE_F64_FN(never)

    def comm(self, n_global):
        return _lib.EbtComm(self.rank, self.world, n_global, self._fn, None, self._ar)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--sample", type=int, default=16)
    ap.add_argument("--replay", type=int, default=0,
                    help="then rank 0 alone replays this many steps (three batches in flight), "
                         "every all-gather answered from the recording of the threaded run: "
                         "rank 0's whole per-rank step at C5/8's real shard size, "
                         "communication excluded")
    a = ap.parse_args()
    cfg = bench.CONFIGS["C5"]
    W, k, B, N = a.world, cfg["k"], cfg["b"], cfg["n"]
    dev = torch.device("cuda:0")
    ebt.load()
    t0 = time.perf_counter()
    cats = []
    for r in range(W):
        b0, b1 = shard_range(N, r, W)
        cats.append(ebt.Catalog(bench.make_catalog_shard(cfg, b0, b1, dev), row_offset=b0,
                                n_global=N))
        torch.cuda.synchronize()
        log(f"shard {r}: rows [{b0}, {b1}), {torch.cuda.memory_allocated() / 2**30:.1f} GiB "
            "allocated")
    q = bench.make_queries(cfg, dev)
    shared = {"slots": [None] * W, "barrier": threading.Barrier(W, timeout=900), "record": []}
    outs, errs = [None] * W, []
    engs = [None] * W
    ws_gib = []

    def rank_body(r):
        try:
            def gather(recv, send):
                n = send.numel()
                shared["slots"][r] = send.clone()
                torch.cuda.current_stream().synchronize()
                shared["barrier"].wait()
                for i in range(W):
                    recv[i * n:(i + 1) * n].copy_(shared["slots"][i])
                torch.cuda.current_stream().synchronize()
                shared["barrier"].wait()
                if r == 0 and a.replay:
                    shared["record"].append(recv.clone())
            engs[r] = ShardedTopk(cats[r], k, B, _AllReduceSlot(r, W, gather=gather), slots=1)
            if r == 0:
                ws_gib.append(engs[r].ws_bytes / 2**30)
            shared["barrier"].wait()      # every rank's workspace allocated before any step
            s, rr = engs[r](queries=q)
            outs[r] = (s.clone(), rr.clone())
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            shared["barrier"].abort()
    t1 = time.perf_counter()
    ts = [threading.Thread(target=rank_body, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    torch.cuda.synchronize()
    step_s = time.perf_counter() - t1
    peak = torch.cuda.max_memory_allocated() / 2**30
    log(f"8 thread ranks done in {step_s:.1f} s (time-shared GPU), peak {peak:.1f} GiB")
    s0, r0 = outs[0]
    same = all(torch.equal(outs[i][1], r0) and
               torch.equal(outs[i][0].nan_to_num(-9.0), s0.nan_to_num(-9.0)) for i in range(W))
    del engs[:]
    torch.cuda.empty_cache()
    # properties of every query: sorted (score desc, row asc), distinct rows, in range
    rr = r0.cpu().numpy()
    ss = s0.cpu().numpy()
    valid = rr >= 0
    props = bool(valid.all() and (rr < N).all() and
                 all(len(np.unique(x)) == k for x in rr[:256]) and
                 bool(np.all((ss[:, :-1] > ss[:, 1:]) | ((ss[:, :-1] == ss[:, 1:]) &
                                                        (rr[:, :-1] < rr[:, 1:])))))
    # sampled queries vs the host float64 oracle over all 50M rows (streamed from the shards)
    idx = np.unique(np.linspace(0, B - 1, a.sample).round().astype(np.int64))
    qh = q[torch.from_numpy(idx).to(dev)].float().cpu().numpy()

    def blocks(block=1 << 18):
        nb = 0
        for c in cats:
            for lo in range(0, c.n, block):
                hi = min(lo + block, c.n)
                nb += 1
                if nb % 20 == 0:   # progress (a silent run longer than 3 minutes reads as hung)
                    log(f"oracle: {c.row_offset + hi} of {N} rows")
                yield c.row_offset + lo, c.data[lo:hi].float().cpu().numpy()
    log(f"host float64 oracle on {len(idx)} queries over {N} rows")
    t2 = time.perf_counter()
    s_o, r_o = R.cosine_topk_stream(qh, blocks(), k, None, workers=8)
    log(f"oracle done in {time.perf_counter() - t2:.0f} s")
    rows_exact = bool(np.array_equal(rr[idx], r_o))
    dmax = float(np.max(np.abs(ss[idx] - s_o)))
    replay = None
    if a.replay:
        # rank 0 alone: the other shards freed, three workspaces, every all-gather replayed
        record = shared["record"]
        by_size = {}
        for g in record:   # one batch's gathers, by size: with batches in flight the floor
            by_size.setdefault(g.numel(), []).append(g)   # and results gathers interleave
        cat0 = cats[0]
        del cats[1:]
        torch.cuda.empty_cache()
        state = {"i": 0, "n": {}}

        def rgather(recv, send):
            lst = by_size[recv.numel()]
            j = state["n"].get(recv.numel(), 0)
            state["n"][recv.numel()] = j + 1
            recv.copy_(lst[j % len(lst)])
        timer = ebt.Timer()
        eng = ShardedTopk(cat0, k, B, _AllReduceSlot(0, W, gather=rgather), slots=3, timer=timer)
        eng.run(1, q)                      # warm
        torch.cuda.synchronize()
        state["n"] = {}
        timer.reset()
        t3 = time.perf_counter()
        s1, r1 = eng.run(a.replay, q)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t3) * 1e3 / a.replay
        from robot_ebert_amd._lib import STAGES
        st = {n: round(timer.query(n)[0] / a.replay, 3) for n in STAGES}
        replay = {"steps": a.replay, "wall_ms_per_step": round(wall, 2),
                  "equals_threaded_run": bool(torch.equal(r1, r0)),
                  "gathers_per_step": len(record),
                  "received_mb_per_step": round(sum(g.numel() for g in record) / 1e6, 1),
                  "stages_ms_per_step": st}
        log(f"replay: {wall:.1f} ms per step")
    print(json.dumps({
        "what": "C5 (50M x 1536 f16, 16384 queries, top-1000) on 8 thread ranks of 6.25M-row "
                "shards, one MI355X, one batch through ebt_cosine_topk_sharded_* (C ABI), "
                "barrier all-gathers between the threads",
        "world": W, "shard_rows": shard_range(N, 0, W)[1], "batch": B, "k": k,
        "workspace_gib_per_rank_slot": round(ws_gib[0], 2) if ws_gib else None,
        "peak_allocated_gib": round(peak, 1), "step_s_all_ranks_time_shared": round(step_s, 1),
        "ranks_agree": same, "properties_ok": props,
        "oracle_queries": int(len(idx)), "rows_bit_exact": rows_exact,
        "max_abs_score_diff": dmax, "setup_s": round(t1 - t0, 1),
        "rank0_replay": replay}), flush=True)
    if not (same and props and rows_exact and dmax <= 1e-5) or (
            replay is not None and not replay["equals_threaded_run"]):
        sys.exit(1)


if __name__ == "__main__":
    main()
