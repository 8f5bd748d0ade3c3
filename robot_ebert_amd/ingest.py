"""Catalog ingest: from the reference's storage formats to an HBM ``Catalog``.

The reference builds its catalog at import time from Chroma (``src/backend/app/constants.py:55-56``):
``collection.get(include=["embeddings"])`` -> ``DataFrame(data=embeddings, index=ids)`` (float64,
rows in Chroma's order, string tmdb ids). ``lib.py:55-62`` then relies on LEXICOGRAPHIC id order
(``sort_index`` on a str index, ``ORDER BY tmdb_id``). These helpers keep both contracts: rows stay
in the source order (so row r here is row r of the reference DataFrame) and ``id_order`` gives the
string order used for pairing.
"""
from __future__ import annotations

from typing import Mapping, Optional, Sequence, Tuple

import numpy as np

from ._lib import EbertError


def chroma_matrix(got: Mapping) -> Tuple[list, np.ndarray]:
    """(ids, float64 [n, d] matrix) of a ``collection.get(include=["embeddings"])`` result, in
    its order -- exactly the DataFrame of constants.py:55-56."""
    if "ids" not in got or "embeddings" not in got or got["embeddings"] is None:
        raise EbertError("need a collection.get(include=['embeddings']) result with ids")
    ids = [str(i) for i in got["ids"]]
    emb = np.asarray(got["embeddings"], dtype=np.float64)
    if emb.ndim != 2 or emb.shape[0] != len(ids):
        raise EbertError(f"{len(ids)} ids for an embeddings array of shape {emb.shape}")
    if len(set(ids)) != len(ids):
        raise EbertError("duplicate ids in the collection")
    return ids, np.ascontiguousarray(emb)


def id_order(ids: Sequence[str]) -> np.ndarray:
    """Row permutation sorting the string ids lexicographically (pandas ``sort_index`` on a str
    index, SQL ``ORDER BY tmdb_id``): ``ids[id_order(ids)]`` is the order lib.py:55-62 pairs in."""
    return np.array(sorted(range(len(ids)), key=lambda i: ids[i]), dtype=np.int64)


def catalog_from_chroma(got: Mapping, device="cuda", dtype=None, shard: bool = False):
    """HBM catalog of a Chroma ``collection.get`` result (float64 like the reference, or
    ``dtype`` -- e.g. torch.float32 -- to store it narrower; the exact rescore then runs on that
    representation)."""
    import torch
    from .catalog import Catalog
    ids, emb = chroma_matrix(got)
    t = torch.from_numpy(emb)
    if dtype is not None:
        t = t.to(dtype)
    return Catalog.from_matrix(ids, t, device=device, shard=shard)


def catalog_from_dataframe(df, device="cuda", dtype=None, shard: bool = False):
    """HBM catalog of a ``DataFrame(index=ids)`` like ``movies_collab_embeddings``."""
    return catalog_from_chroma({"ids": list(df.index), "embeddings": df.values}, device=device,
                               dtype=dtype, shard=shard)
