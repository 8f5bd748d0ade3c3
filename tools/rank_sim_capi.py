"""Rank 0 of an N-rank bench.py run through the C ABI's pipelined sharded step
(distributed.ShardedTopk over ebt_cosine_topk_sharded_submit / _finish / _wait) in ONE process on
one MI355X, every all-gather answered from a recording -- the C-path twin of tools/rank_sim.py.

First all N ranks run the steps as threads (the all-gather by barrier exchange through a
TorchGatherComm callback) while rank 0's gathered buffers are recorded in call order; then rank 0
replays the identical steps alone, each all-gather copying the recorded buffer into place. Reports
  * wall_ms_per_step: rank 0's pipelined step (three batches in flight), communication excluded;
  * host_ms_per_step: the host work of one step (submit + finish + wait), measured with the GPU
    drained before each call, so no call waits for the GPU; callback_ms_per_step is the part
    spent in the replay's Python all-gather callback (RCCL's ncclAllGather enqueue replaces it
    on a real node);
  * exchange bytes per rank and step (what each all-gather receives), and the per-stage GPU time.

    python tools/rank_sim_capi.py [--config C3] [--world 8] [--steps 20]
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import _lib  # noqa: E402
from robot_ebert_amd.distributed import ShardedTopk, TorchGatherComm, shard_range  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    ebt.load()
    W, k, B = a.world, cfg["k"], cfg["b"]
    cats = []
    for r in range(W):
        b0, b1 = shard_range(cfg["n"], r, W)
        cats.append(ebt.Catalog(bench.make_catalog_shard(cfg, b0, b1, dev), row_offset=b0,
                                n_global=cfg["n"]))
        torch.cuda.synchronize()
        print(f"shard {r}: rows [{b0}, {b1})", file=sys.stderr, flush=True)
    q = bench.make_queries(cfg, dev)
    shared = {"slots": [None] * W, "barrier": threading.Barrier(W, timeout=300), "record": []}
    outs = [None] * W
    errs = []

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
                if r == 0:
                    shared["record"].append(recv.clone())
            comm = TorchGatherComm(r, W, gather=gather)
            eng = ShardedTopk(cats[r], k, B, comm)
            s, rr = eng.run(a.steps, q)
            outs[r] = (s.clone(), rr.clone())
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            shared["barrier"].abort()
    ts = [threading.Thread(target=rank_body, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    torch.cuda.synchronize()
    print("thread ranks done", file=sys.stderr, flush=True)
    record = shared["record"]
    per_step = len(record) // a.steps
    sizes = sorted(set(int(g.numel()) for g in record))
    recv_total = sum(int(g.numel()) for g in record)
    # the packed results' gathers: every rank's entries above the floor = the sum of its
    # per-query len[B] (header u32 start[B], u32 len[B] since ABI 0.3.2)
    lib = _lib.load()
    w = int(lib.ebt_shard_list_width(k, W))
    cap = int(lib.ebt_shard_pack_cap(B, k, W, cfg["n"]))
    pb = int(lib.ebt_shard_pack_bytes(B, cap)) if cap else 0
    counts = []
    for g in record:
        if pb and g.numel() == W * pb:
            v = g.view(W, pb)[:, :8 * B].contiguous().view(torch.int32)
            counts.append(v[:, B:2 * B].double().sum(1).cpu())
    sent = torch.stack(counts) if counts else None
    ref = outs[0]
    cat0 = cats[0]
    del cats[1:]
    torch.cuda.empty_cache()

    state = {"i": 0, "cb_s": 0.0}

    def replay(recv, send):
        t0 = time.perf_counter()
        g = record[state["i"] % len(record)]
        state["i"] += 1
        assert g.numel() == recv.numel(), (g.numel(), recv.numel())
        recv.copy_(g)
        state["cb_s"] += time.perf_counter() - t0

    comm = TorchGatherComm(0, W, gather=replay)
    timer = ebt.Timer()
    eng = ShardedTopk(cat0, k, B, comm, timer=timer)
    timer.only("gemm_filter")

    def rerun():
        state["i"] = 0
        return eng.run(a.steps, q)
    rerun()   # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s, r = rerun()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / a.steps
    same = bool(torch.equal(r, ref[1]) and torch.equal(s.nan_to_num(-9.0), ref[0].nan_to_num(-9.0)))

    # host work per step: each call made with the GPU drained (no call waits for the GPU)
    state["i"], state["cb_s"] = 0, 0.0
    host = {"submit": 0.0, "finish": 0.0, "wait": 0.0}
    S = 3
    for i in range(a.steps + 2):
        for name, cond, fn in (("submit", i < a.steps, lambda: eng.submit(i % S, queries=q)),
                               ("finish", 1 <= i <= a.steps, lambda: eng.finish((i - 1) % S)),
                               ("wait", i >= 2, lambda: eng.wait((i - 2) % S))):
            if not cond:
                continue
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            fn()
            host[name] += time.perf_counter() - t1
    torch.cuda.synchronize()
    host_ms = {n: round(v * 1e3 / a.steps, 4) for n, v in host.items()}
    cb_ms = state["cb_s"] * 1e3 / a.steps

    timer.only()
    timer.reset()
    rerun()
    torch.cuda.synchronize()
    stages = {n: round(timer.query(n)[0] / a.steps, 4) for n in _lib.STAGES}
    print(json.dumps({
        "config": a.config, "world": W, "shard_rows": cat0.n, "path": "C ABI (ShardedTopk)",
        "gathers_per_step": per_step, "gather_sizes_bytes": sizes,
        "recv_mb_per_step": round(recv_total / a.steps / 1e6, 3),
        "floor_width_per_query": w, "packed_cap_per_rank": cap, "packed_bytes_per_rank": pb,
        "packed_entries_per_query_mean": (round(float(sent.mean()) / B, 2)
                                          if sent is not None else None),
        "packed_entries_per_query_max_rank": (round(float(sent.max()) / B, 2)
                                              if sent is not None else None),
        "wall_ms_per_step": round(wall, 3), "replay_equals_threads": same,
        "host_ms_per_step": round(sum(host_ms.values()), 4), "host_ms_by_call": host_ms,
        "callback_ms_per_step": round(cb_ms, 4),
        "host_ms_excl_callback": round(sum(host_ms.values()) - cb_ms, 4),
        "stages_ms_per_step_timed_run": stages,
        "stage_sum_ms": round(sum(stages.values()), 3)}), flush=True)


if __name__ == "__main__":
    main()
