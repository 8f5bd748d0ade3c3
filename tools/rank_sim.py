"""Rank 0 of an N-rank bench.py run in ONE process on one MI355X: the full N > 1 Python pipeline
(distributed.run_sharded_steps over score_topk_sharded_local_stages: shared threshold, floor,
per-shard rescore, results all-gather, merge) on rank 0's shard, with every all-gather answered
from a recording. First all N ranks run the same steps as threads on the GPU (collectives by
barrier exchange) while rank 0's gathered tensors are recorded in call order; then rank 0 runs
the identical steps alone and each all-gather returns (a device copy of) the recorded tensor.
So rank 0 does exactly its real work, minus the communication: wall time per step vs the GPU's
busy time says whether the host keeps ahead of the GPU at the 8-way step.

    python tools/rank_sim.py [--config C3] [--world 8] [--steps 20]
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
from robot_ebert_amd.distributed import (run_sharded_steps,  # noqa: E402
                                         score_topk_sharded_local_stages, shard_range)


class RecordingCollectives:
    """Thread ranks exchanging through a barrier; rank 0 records every gathered tensor."""

    def __init__(self, rank, shared):
        self.rank, self.s, self.world = rank, shared, shared["world"]

    def all_gather(self, t):
        self.s["slots"][self.rank] = t.clone()
        self.s["barrier"].wait()
        g = torch.stack(list(self.s["slots"]))
        self.s["barrier"].wait()
        if self.rank == 0:
            self.s["record"].append(g)
        return g

    def all_gather_start(self, t):
        g = self.all_gather(t)
        return lambda: g


class ReplayCollectives:
    def __init__(self, world, record):
        self.world, self.rank, self.rec, self.i = world, 0, record, 0

    def all_gather(self, t):
        g = self.rec[self.i % len(self.rec)]
        self.i += 1
        assert g.shape[1:] == t.shape and g.dtype == t.dtype, (g.shape, t.shape)
        return g.clone()

    def all_gather_start(self, t):
        g = self.all_gather(t)
        return lambda: g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--profile", action="store_true",
                    help="also cProfile the replayed steps (host time by function, to stderr)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    ebt.load()
    W, k = a.world, cfg["k"]
    cats = []
    for r in range(W):
        b0, b1 = shard_range(cfg["n"], r, W)
        cats.append(ebt.Catalog(bench.make_catalog_shard(cfg, b0, b1, dev), row_offset=b0,
                                n_global=cfg["n"]))
        torch.cuda.synchronize()
        print(f"shard {r}: rows [{b0}, {b1})", file=sys.stderr, flush=True)
    q = bench.make_queries(cfg, dev)
    shared = {"world": W, "slots": [None] * W, "barrier": threading.Barrier(W, timeout=300),
              "record": []}
    outs = [None] * W

    def rank_body(r):
        coll = RecordingCollectives(r, shared)
        outs[r] = run_sharded_steps(
            lambda: score_topk_sharded_local_stages(cats[r], k, queries=q, collectives=coll),
            a.steps)
    ts = [threading.Thread(target=rank_body, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    print("thread ranks done", file=sys.stderr, flush=True)
    record = shared["record"]
    per_step = len(record) // a.steps if a.steps else 0
    ref = outs[0]
    cat0 = cats[0]
    del cats[1:]
    torch.cuda.empty_cache()

    def run(tm=None):
        coll = ReplayCollectives(W, record)
        return run_sharded_steps(
            lambda: score_topk_sharded_local_stages(cat0, k, queries=q, collectives=coll,
                                                    timer=tm), a.steps)
    run()   # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s, r = run()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / a.steps
    same = bool(torch.equal(r, ref[1]) and torch.equal(s.nan_to_num(-9.0), ref[0].nan_to_num(-9.0)))
    if a.profile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        run()
        torch.cuda.synchronize()
        pr.disable()
        st = pstats.Stats(pr, stream=sys.stderr)
        st.sort_stats("tottime").print_stats(30)
        st.sort_stats("cumulative").print_stats(40)
    timer = ebt.Timer()
    run(timer)
    torch.cuda.synchronize()
    stages = {n: round(timer.query(n)[0] / a.steps, 4) for n in _lib.STAGES}
    out = {"config": a.config, "world": W, "shard_rows": cat0.n,
           "gathers_recorded": len(record), "gathers_per_step": per_step,
           "recv_mb_per_step": round(sum(g.numel() * g.element_size() for g in record)
                                     / a.steps / 1e6, 3),
           "wall_ms_per_step": round(wall, 3), "replay_equals_threads": same,
           "stages_ms_per_step_timed_run": stages,
           "stage_sum_ms": round(sum(stages.values()), 3)}
    if record[-1].dtype == torch.uint8:   # the packed results exchange (merge_packed)
        print(json.dumps(out), flush=True)
        return
    # the post-gather merge alone on the last recorded results (the last two gathers)
    from robot_ebert_amd.search import merge_topk
    gs, gr = record[-2], record[-1]
    merge_topk(gs, gr, k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        merge_topk(gs, gr, k)
    e1.record()
    torch.cuda.synchronize()
    merge_alone = e0.elapsed_time(e1) / 10
    # the gathered lists: sorted (score desc, row asc)? candidates of the co-rank merge (entries
    # up to m0 = the last of the lists' ceil(k/R)-th entries)
    sc_, rw_ = gs.double().cpu(), gr.cpu()
    nxt_before = (sc_[:, :, 1:] > sc_[:, :, :-1]) | ((sc_[:, :, 1:] == sc_[:, :, :-1]) &
                                                     (rw_[:, :, 1:] < rw_[:, :, :-1]))
    unsorted_lists = int(nxt_before.any(2).sum())
    kr = -(-k // W)
    m0 = sc_[:, :, kr - 1].min(0).values                       # [B] (ties by row ignored)
    cands = (sc_ >= m0[None, :, None]).sum((0, 2)).double()
    diag = {"unsorted_lists": unsorted_lists, "lists": W * sc_.shape[1],
            "candidates_mean": round(float(cands.mean()), 1),
            "candidates_max": int(cands.max())}
    out.update(merge_alone_ms=round(merge_alone, 4), merge_lists=diag)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
