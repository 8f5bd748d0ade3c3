"""Per-rank compute of the sharded paths at N ranks, on ONE GPU: N threads, one per simulated
rank, each with its own shard of the C3 catalog, exchanging through in-process collectives (no
communication cost). The GPU runs the ranks' work back to back, so per-rank time ~ the step
time / N. Compares the two-phase path with the per-shard-rescore path.

    python tools/shard_sim.py [--config C3] [--ranks 2 4 8] [--steps 3] [--one-rank]
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
from robot_ebert_amd.distributed import score_topk_sharded, shard_range  # noqa: E402


class ThreadCollectives:
    def __init__(self, rank, shared):
        self.rank, self.s, self.world = rank, shared, shared["world"]

    def _exchange(self, t):
        self.s["slots"][self.rank] = t.clone()
        self.s["barrier"].wait()
        vals = list(self.s["slots"])
        self.s["barrier"].wait()
        return vals

    def all_gather(self, t):
        return torch.stack(self._exchange(t))

    def all_reduce_sum(self, t):
        t.copy_(torch.stack(self._exchange(t)).sum(0))
        return t

    def all_reduce_max(self, t):
        t.copy_(torch.stack(self._exchange(t)).max(0).values)
        return t


def one_rank(args):
    """Per-rank GPU time of score_topk_sharded_local without thread contention: every shard's
    floor (approx[k-1] - eps) is computed first, then rank 0 runs alone with the all-reduce
    replaced by the stored max."""
    from robot_ebert_amd import _lib, search
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda:0")
    q = bench.make_queries(cfg, dev)
    k = cfg["k"]
    from robot_ebert_amd.distributed import (local_sample, shared_sample_tiles,
                                             theta_from_samples)
    for R in args.ranks:
        floors, samples = [], []
        cat0 = None
        tiles = shared_sample_tiles(cfg["n"], R, search.pad_batch(q.shape[0]))
        for r in range(R):
            a, b = shard_range(cfg["n"], r, R)
            cat = ebt.Catalog(bench.make_catalog_shard(cfg, a, b, dev), row_offset=a,
                              n_global=cfg["n"])
            qb = search.prepare_queries(cat, queries=q)
            kp = search.default_kprime(cat, k)
            lv, _, _, eps = search.run_screen(cat, qb, k, kp)
            floors.append((lv[:, :k].clone(), eps[:qb.B].clone()))
            if tiles:
                samples.append(local_sample(cat, qb, tiles))
            if r == 0:
                cat0, lv0, eps0 = cat, lv.double(), eps[:qb.B].double()
            else:
                del cat
            torch.cuda.empty_cache()
        t_glob = search.union_floor(torch.stack([f[0] for f in floors]),
                                    torch.stack([f[1] for f in floors]), k)
        cut0 = lv0[:, k - 1] - 2 * eps0
        cut1 = torch.maximum(cut0, t_glob - eps0)
        print(json.dumps({"ranks": R, "kprime": lv0.shape[1],
                          "eps_mean": float(eps0.mean()),
                          "kth_minus_first_mean": float((lv0[:, 0] - lv0[:, k - 1]).mean()),
                          "rescored_nocut": float((lv0 >= cut0[:, None]).sum(1).double().mean()),
                          "rescored_cut": float((lv0 >= cut1[:, None]).sum(1).double().mean())}),
              flush=True)
        variants = [("cut", lambda v, e: t_glob.clone(), None), ("nocut", None, None)]
        if tiles:  # rank 0 screened at the catalog-wide threshold of all shards' samples
            g = torch.stack(samples)
            variants.insert(0, ("shared", lambda v, e: t_glob.clone(),
                                lambda qb, kp: theta_from_samples(g, qb, kp, tiles, cfg["n"],
                                                                  cat0.n)))
            qb0 = search.prepare_queries(cat0, queries=q)
            th, hits = theta_from_samples(g, qb0, search.default_kprime(cat0, k), tiles,
                                          cfg["n"], cat0.n)
            fails = int((th[:qb0.B].double() > t_glob - eps0).sum())
            print(json.dumps({"ranks": R, "shared_tiles": tiles, "expected_hits": round(hits, 1),
                              "theta_failures": fails}), flush=True)
        if args.only:
            variants = [v for v in variants if v[0] == args.only]
        ref = None
        for name, hook, th_hook in variants:
            pending = None  # pipelined as bench.py does: submit step i+1, then finish step i
            for i in range(args.steps + 1):
                if i == 1:
                    search.score_topk_finish(pending)
                    pending = None
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                p = search.score_topk_submit(cat0, k, queries=q, t_floor_hook=hook,
                                             theta_hook=th_hook)
                if pending is not None:
                    search.score_topk_finish(pending)
                pending = p
            search.score_topk_finish(pending)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            tm = ebt.Timer()
            s_, r_ = search.score_topk(cat0, k, queries=q, t_floor_hook=hook, theta_hook=th_hook,
                                       timer=tm)
            torch.cuda.synchronize()
            same = None
            if name == "shared" or ref is not None:
                if ref is None:
                    ref = (s_, r_)
                else:
                    same = bool(torch.equal(r_, ref[1]) and torch.allclose(s_, ref[0], rtol=0, atol=0,
                                                                           equal_nan=True))
            print(json.dumps({"config": args.config, "ranks": R, "path": "one_rank_" + name,
                              "ms_per_step": round(ms, 3),
                              "same_as_shared": same,
                              "stages_ms": {kk: round(tm.query(kk)[0], 3) for kk in _lib.STAGES}}),
                  flush=True)
        del cat0
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--one-rank", action="store_true",
                    help="time rank 0's own work alone (the floor all-reduce replaced by its "
                         "precomputed result) with and without the global cut")
    ap.add_argument("--only", default=None, choices=["shared", "cut", "nocut"],
                    help="--one-rank: time only this variant (profiling)")
    args = ap.parse_args()
    if args.one_rank:
        return one_rank(args)
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda:0")
    q = bench.make_queries(cfg, dev)
    import threading
    from robot_ebert_amd.distributed import score_topk_sharded_local
    for R in args.ranks:
        cats = []
        for r in range(R):
            a, b = shard_range(cfg["n"], r, R)
            cats.append(ebt.Catalog(bench.make_catalog_shard(cfg, a, b, dev), row_offset=a,
                                    n_global=cfg["n"]))
        def per_shard_nocut(*a, **kw):
            return score_topk_sharded_local(*a, t_floor_hook=None, **kw)
        for name, fn in (("two_phase", score_topk_sharded), ("per_shard", score_topk_sharded_local),
                         ("per_shard_nocut", per_shard_nocut)):
            shared = {"world": R, "slots": [None] * R, "barrier": threading.Barrier(R)}

            def rank_body(r):
                coll = ThreadCollectives(r, shared)
                for _ in range(args.steps + 1):
                    fn(cats[r], cfg["k"], queries=q, collectives=coll)
            torch.cuda.synchronize()
            ts = [threading.Thread(target=rank_body, args=(r,)) for r in range(R)]
            t0 = time.perf_counter()
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / (args.steps + 1)
            print(json.dumps({"ranks": R, "path": name, "gpu_ms_per_step_all_ranks": round(ms, 3),
                              "per_rank_ms_estimate": round(ms / R, 3)}), flush=True)
        del cats
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
