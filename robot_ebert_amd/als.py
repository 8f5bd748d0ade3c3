"""Implicit-feedback ALS on the GPU: the offline training of the collaborative catalog that the
recommend path serves.

The reference trains it with Spark (notebooks/create-embeddings.ipynb:1055):
    ALS(rank=32, maxIter=15, regParam=0.1, implicitPrefs=True, userCol='user_id',
        itemCol='tmdb_id', ratingCol='rating')
then upserts the item factors into Chroma (`:1250`), where constants.py:55-56 reads them as the
catalog. Here every half-iteration is two HIP kernels (csrc/als.hip): the float64 gram Y^T Y and
one workgroup per destination building and solving its normal equation (Spark's
computeFactors, implicit branch: float64 accumulation and Cholesky, float32 factors). The
result feeds `Catalog.from_matrix` / `ingest.catalog_from_dataframe` directly.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ._lib import EbertError, call, ptr, stream_of


class Ratings:
    """A ratings matrix on the device in both CSR orientations (by user and by item)."""

    def __init__(self, users, items, ratings, n_users: int, n_items: int, device) -> None:
        users = np.asarray(users, dtype=np.int64)
        items = np.asarray(items, dtype=np.int64)
        vals = np.asarray(ratings, dtype=np.float32)
        if not (users.shape == items.shape == vals.shape):
            raise EbertError("users, items and ratings must have the same length")
        if users.size and (users.min() < 0 or users.max() >= n_users or items.min() < 0 or
                           items.max() >= n_items):
            raise EbertError("user / item index out of range")
        self.n_users, self.n_items, self.device = int(n_users), int(n_items), device
        self.by_user = self._csr(users, items, vals, n_users)
        self.by_item = self._csr(items, users, vals, n_items)

    def _csr(self, rows, cols, vals, n):
        order = np.lexsort((cols, rows))
        off = np.zeros(n + 1, dtype=np.int64)
        np.add.at(off, rows[order] + 1, 1)
        dev = self.device
        return (torch.from_numpy(np.cumsum(off)).to(dev),
                torch.from_numpy(cols[order].astype(np.int32)).to(dev),
                torch.from_numpy(vals[order]).to(dev))


def gram(Y: torch.Tensor) -> torch.Tensor:
    """ebt_als_gram: Y^T Y in float64 ([rank, rank]) of float32 factors Y [n, rank]."""
    Y = Y.contiguous()
    out = torch.empty((Y.shape[1], Y.shape[1]), dtype=torch.float64, device=Y.device)
    call("ebt_als_gram", ptr(Y), Y.shape[0], Y.shape[1], ptr(out), stream_of(Y.device))
    return out


def half_step(Y: torch.Tensor, csr, alpha: float, reg: float) -> torch.Tensor:
    """Every destination factor from the source factors Y (ebt_als_solve)."""
    off, src, val = csr
    Y = Y.contiguous()
    X = torch.empty((off.numel() - 1, Y.shape[1]), dtype=torch.float32, device=Y.device)
    YtY = gram(Y)
    call("ebt_als_solve", ptr(YtY), ptr(Y), Y.shape[1], X.shape[0], ptr(off), ptr(src), ptr(val),
         float(alpha), float(reg), ptr(X), stream_of(Y.device))
    return X


def init_factors(n: int, rank: int, seed: int, device) -> torch.Tensor:
    """Random unit-norm float32 rows (Spark's scheme: Gaussian entries, each row normalised;
    Spark's own RNG stream is not reproduced)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn((n, rank), generator=g, dtype=torch.float64)
    x = x / x.norm(dim=1, keepdim=True).clamp_min(1e-300)
    return x.to(torch.float32).to(device)


def train(ratings: Ratings, rank: int = 32, iters: int = 15, reg: float = 0.1,
          alpha: float = 1.0, seed: int = 0, U0: Optional[torch.Tensor] = None,
          V0: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """ALS(rank, maxIter=iters, regParam=reg, implicitPrefs=True, alpha): (user factors,
    item factors), float32 on the ratings' device. Each iteration recomputes the items from
    the users, then the users from the items (Spark's order)."""
    if not ratings.device.type == "cuda":
        raise EbertError("ALS runs on the GPU (libebert has no CPU path)")
    dev = ratings.device
    U = U0.to(dev, torch.float32) if U0 is not None else init_factors(ratings.n_users, rank,
                                                                     seed, dev)
    V = V0.to(dev, torch.float32) if V0 is not None else init_factors(ratings.n_items, rank,
                                                                     seed + 1, dev)
    for _ in range(iters):
        V = half_step(U, ratings.by_item, alpha, reg)
        U = half_step(V, ratings.by_user, alpha, reg)
    return U, V
