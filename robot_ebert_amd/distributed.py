"""Row-sharded catalog over the GPUs of one node (one process per GPU, torch.distributed).

The reference scales only by Cloud Run replicas (README.md:78-82) and has no collective. Here
the catalog rows are split into contiguous blocks, rank r holding rows
[shard_range(n, r, R)), and every rank scores the full query batch against its shard (global row
ids via ``row_offset``). The ONE exchange step is an all-gather of the per-shard top-k
(B x k float64 scores + B x k int64 rows, a few MB) over RCCL/xGMI, followed by the
``ebt_merge_topk`` kernel on every rank. For the collaborative path the liked rows of a user live
on several shards: each rank sums its local normalised liked rows and one all-reduce (SUM) of the
B x d float64 partial sums completes the query vectors before screening.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .catalog import Catalog
from .search import csr_from_lists, merge_topk, score_topk


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block of rows owned by `rank` (sizes differ by at most one row)."""
    base, rem = divmod(n, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def gather_partials(scores: torch.Tensor, rows: torch.Tensor,
                    group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather the [B, k] partial results of every rank -> [R, B, k] (rank order)."""
    world = dist.get_world_size(group)
    B = scores.shape[0]
    # concatenated along dim 0 (the layout every backend accepts), viewed as [R, B, k]
    gs = torch.empty((world * B,) + tuple(scores.shape[1:]), dtype=scores.dtype,
                     device=scores.device)
    gr = torch.empty((world * B,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(gs, scores.contiguous(), group=group)
    dist.all_gather_into_tensor(gr, rows.contiguous(), group=group)
    return gs.view((world,) + tuple(scores.shape)), gr.view((world,) + tuple(rows.shape))


def split_liked(liked: Sequence[Sequence[int]], begin: int, end: int):
    """Per-user liked rows that fall into [begin, end), plus every user's total count."""
    local = [[r for r in l if begin <= r < end] for l in liked]
    counts = [len(l) for l in liked]
    return local, counts


def score_topk_sharded(catalog: Catalog, k: int, queries: Optional[torch.Tensor] = None,
                       liked: Optional[Sequence[Sequence[int]]] = None,
                       exclude=None, group: Optional[dist.ProcessGroup] = None,
                       **kw) -> Tuple[torch.Tensor, torch.Tensor]:
    """Global top-k over a row-sharded catalog; every rank returns the same [B, k] result."""
    dev = catalog.device
    hook = None
    liked_arg = None
    counts_t = None
    if liked is not None:
        local, counts = split_liked(liked, catalog.row_offset, catalog.row_offset + catalog.n)
        liked_arg = csr_from_lists(local, dev)
        counts_t = torch.tensor(counts, dtype=torch.int64, device=dev)

        def hook(q64: torch.Tensor) -> torch.Tensor:
            dist.all_reduce(q64, op=dist.ReduceOp.SUM, group=group)
            return q64

    s, r = score_topk(catalog, k, queries=queries, liked=liked_arg, exclude=exclude,
                      liked_counts=counts_t, liked_sum_hook=hook, **kw)
    gs, gr = gather_partials(s, r, group)
    return merge_topk(gs, gr, k)
