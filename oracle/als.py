"""TEST INFRASTRUCTURE ONLY -- float64 numpy restatement of implicit-feedback ALS as the reference
trains its collaborative embeddings (notebooks/create-embeddings.ipynb:1055:
pyspark.ml.recommendation.ALS(rank=32, maxIter=15, regParam=0.1, implicitPrefs=True), alpha at
its default 1.0). Only tests/ and tools/ may import it; the product path is
robot_ebert_amd/als.py over the HIP kernels of csrc/als.hip.

The algorithm is Spark's published one (mllib ALS.scala, computeFactors, implicit branch --
Spark is not installed here, so this restatement is "parity unpinned" against Spark itself):
  YtY = Y^T Y
  for every destination u with ratings (i, r):
      A = YtY + sum_i c1 y_i y_i^T           c1 = alpha |r|
      b = sum_{i: r > 0} (1 + c1) y_i
      x_u = solve(A + reg * n_pos(u) I, b)    (Cholesky, float64)
  factors stored as float32; one iteration = items from users, then users from items
  (ALS.train: itemFactors = computeFactors(userFactors, ...), then userFactors = ...).
Spark's random initialisation (its own RNG) is not restated: both sides start from the same
given factors.
"""
from __future__ import annotations

import numpy as np


def half_step(Y: np.ndarray, off: np.ndarray, src: np.ndarray, rating: np.ndarray,
              alpha: float, reg: float) -> np.ndarray:
    """Recompute every destination factor from source factors Y (float32 [n_src, rank])."""
    Y64 = Y.astype(np.float64)
    rank = Y.shape[1]
    YtY = Y64.T @ Y64
    n_dst = len(off) - 1
    X = np.zeros((n_dst, rank), dtype=np.float32)
    for u in range(n_dst):
        s, e = int(off[u]), int(off[u + 1])
        ys = Y64[src[s:e]]
        r = rating[s:e].astype(np.float64)
        c1 = alpha * np.abs(r)
        A = YtY + (ys * c1[:, None]).T @ ys
        pos = r > 0
        b = ((1.0 + c1[pos])[:, None] * ys[pos]).sum(0) if pos.any() else np.zeros(rank)
        A[np.diag_indices(rank)] += reg * float(pos.sum())
        L = np.linalg.cholesky(A)
        z = np.linalg.solve(L, b)
        X[u] = np.linalg.solve(L.T, z).astype(np.float32)
    return X


def csr(rows: np.ndarray, cols: np.ndarray, vals: np.ndarray, n_rows: int):
    """COO -> CSR (off int64 [n_rows + 1], cols int32, vals float32), row-major order."""
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    off = np.zeros(n_rows + 1, dtype=np.int64)
    np.add.at(off, rows + 1, 1)
    return np.cumsum(off), cols.astype(np.int32), vals.astype(np.float32)


def train(users: np.ndarray, items: np.ndarray, ratings: np.ndarray, n_users: int, n_items: int,
          U0: np.ndarray, V0: np.ndarray, iters: int, alpha: float = 1.0, reg: float = 0.1):
    """`iters` ALS iterations from the given float32 factors; returns (U, V)."""
    by_user = csr(users, items, ratings, n_users)
    by_item = csr(items, users, ratings, n_items)
    U, V = U0.astype(np.float32), V0.astype(np.float32)
    for _ in range(iters):
        V = half_step(U, *by_item, alpha, reg)
        U = half_step(V, *by_user, alpha, reg)
    return U, V
