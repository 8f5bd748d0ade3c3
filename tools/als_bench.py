"""ALS training throughput on the GPU: ms per iteration (items from
users + users from items) for MovieLens-shaped synthetic ratings, rank 32, reg 0.1, alpha 1, and
the float64 oracle timed on a slice of the smallest shape beside it.

    python tools/als_bench.py
Algorithmic traffic per half-iteration: every rating's source factor (rank x 4 B) + the rating
itself (8 B) + one factor written per destination: reported as GB/s against HBM.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robot_ebert_amd import als  # noqa: E402


def synth(n_users, n_items, n_ratings, seed=0):
    rng = np.random.default_rng(seed)
    # popularity-skewed items (Zipf-like), uniform users, MovieLens rating values
    users = rng.integers(0, n_users, n_ratings)
    items = np.minimum((rng.pareto(1.2, n_ratings) * n_items / 20).astype(np.int64), n_items - 1)
    key = np.unique(users * n_items + items)
    users, items = key // n_items, key % n_items
    vals = rng.choice(np.arange(1, 11) * 0.5, users.size).astype(np.float32)
    return users, items, vals


def main():
    dev = torch.device("cuda:0")
    rank, reg, alpha = 32, 0.1, 1.0
    for name, (nu, ni, nr) in {"ml-latest-small": (610, 9724, 100_836),
                               "ml-25m": (162_541, 59_047, 25_000_095)}.items():
        users, items, vals = synth(nu, ni, nr)
        R = als.Ratings(users, items, vals, nu, ni, dev)
        U, V = als.train(R, rank=rank, iters=1)
        torch.cuda.synchronize()
        iters = 5
        t0 = time.perf_counter()
        U, V = als.train(R, rank=rank, iters=iters, U0=U, V0=V)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / iters
        nnz = users.size
        bytes_it = 2 * (nnz * (rank * 4 + 8)) + (nu + ni) * rank * 4
        out = {"shape": name, "users": nu, "items": ni, "ratings": int(nnz), "rank": rank,
               "ms_per_iter": round(ms, 3), "GBps": round(bytes_it / (ms * 1e-3) / 1e9, 1)}
        if name == "ml-latest-small":
            from oracle import als as O
            by_user = O.csr(users, items, vals, nu)
            Vn = V.cpu().numpy()
            t0 = time.perf_counter()
            O.half_step(Vn, by_user[0][:101], by_user[1], by_user[2], alpha, reg)
            cpu_s = time.perf_counter() - t0
            out["cpu_oracle_users_per_s"] = round(100 / cpu_s, 1)
            out["gpu_users_per_s"] = round(nu / (ms * 1e-3 / 2), 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
