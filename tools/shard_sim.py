"""Per-rank compute of the sharded paths at N ranks, on ONE GPU: N threads, one per simulated
rank, each with its own shard of the C3 catalog, exchanging through in-process collectives (no
communication cost). The GPU runs the ranks' work back to back, so per-rank time ~ the step
time / N. Compares the two-phase path with the per-shard-rescore path.

    python tools/shard_sim.py [--ranks 2 4 8] [--steps 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    cfg = bench.CONFIGS["C3"]
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
        for name, fn in (("two_phase", score_topk_sharded), ("per_shard", score_topk_sharded_local)):
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
