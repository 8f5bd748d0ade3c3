"""PyTorch custom ops over libebert (SURVEY.md §8b "torch op"): the hot path as dispatcher-visible
operators, ``torch.ops.ebert.*``, for callers that hold plain tensors instead of a ``Catalog``.

    gnorm, inv = torch.ops.ebert.row_norms(cat)                 # once per catalog (constants.py:55-56)
    image      = torch.ops.ebert.screen_image(cat, gnorm)       # once per catalog
    s, r = torch.ops.ebert.cosine_topk(q, cat, gnorm, inv, image, k, excl_off, excl_rows, 0)
    s, r = torch.ops.ebert.merge_topk(gathered_s, gathered_r, k) # after an all-gather of shards

Each op is the same libebert call the ``Catalog`` / ``score_topk`` API makes (HIP kernels on the
tensors' device and current stream); nothing is computed in Python or on the CPU. ``cosine_topk``
is ``lib.py:51-55`` for a batch: top-k rows by cosine of each query row against the catalog,
excluded (GLOBAL) rows removed, ordered (score desc, row asc); scores float64, rows int64 GLOBAL
(``row_offset`` + local row), short rows padded with NaN / -1. Fake (meta) kernels give shapes
for tracing.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import DTYPE_CODE, EbertError, call, ptr, require_cuda, stream_of
from .catalog import IMG_ALIGN, Catalog, _round_up


@torch.library.custom_op("ebert::row_norms", mutates_args=())
def row_norms(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Guarded float64 row norms (sklearn _handle_zeros_in_scale) and float32 1/norm padded to
    a multiple of 128 rows (the screening epilogue's row scale)."""
    require_cuda(x, "x")
    if x.dim() != 2 or x.dtype not in DTYPE_CODE:
        raise EbertError("row_norms: x must be a 2-D f32/f64/bf16/f16 CUDA matrix")
    x = x if x.stride(1) == 1 else x.contiguous()
    n, d = x.shape
    g = torch.empty(n, dtype=torch.float64, device=x.device)
    inv = torch.ones(_round_up(n, 128), dtype=torch.float32, device=x.device)
    call("ebt_row_norms", ptr(x), DTYPE_CODE[x.dtype], n, d, int(x.stride(0)), ptr(g), ptr(inv),
         stream_of(x.device))
    return g, inv


@row_norms.register_fake
def _(x):
    n = x.shape[0]
    return (x.new_empty((n,), dtype=torch.float64),
            x.new_empty((_round_up(n, 128),), dtype=torch.float32))


def _image_spec(x: torch.Tensor):
    native = x.dtype in (torch.float16, torch.bfloat16)
    dt = x.dtype if native else torch.float16
    return native, dt, _round_up(x.shape[1], IMG_ALIGN)


@torch.library.custom_op("ebert::screen_image", mutates_args=())
def screen_image(x: torch.Tensor, gnorm: torch.Tensor) -> torch.Tensor:
    """The MFMA operand of a catalog: f16 image of the NORMALISED rows for f32/f64 catalogs, the
    raw rows (a padded copy) for f16/bf16 ones; columns zero-padded to a multiple of 64. (A
    native f16/bf16 catalog whose d is a multiple of 64 can pass itself as the image.)"""
    require_cuda(x, "x")
    require_cuda(gnorm, "gnorm")
    x = x if x.stride(1) == 1 else x.contiguous()
    native, dt, ld = _image_spec(x)
    n, d = x.shape
    img = torch.empty((n, ld), dtype=dt, device=x.device)
    call("ebt_screen_image", ptr(x), DTYPE_CODE[x.dtype], n, d, int(x.stride(0)), ptr(gnorm),
         0 if native else 1, _lib.EBT_F16 if dt == torch.float16 else _lib.EBT_BF16, ptr(img), ld,
         stream_of(x.device))
    return img


@screen_image.register_fake
def _(x, gnorm):
    _, dt, ld = _image_spec(x)
    return x.new_empty((x.shape[0], ld), dtype=dt)


@torch.library.custom_op("ebert::cosine_topk", mutates_args=())
def cosine_topk(q: torch.Tensor, cat: torch.Tensor, gnorm: torch.Tensor, inv: torch.Tensor,
                image: torch.Tensor, k: int, excl_off: Optional[torch.Tensor],
                excl_rows: Optional[torch.Tensor], row_offset: int) -> Tuple[torch.Tensor,
                                                                            torch.Tensor]:
    """Top-k by cosine of each row of q against (a shard of) the catalog, excluded rows dropped
    (lib.py:51-55 for a batch)."""
    from .search import score_topk
    catalog = Catalog.from_parts(cat, gnorm, inv, image, row_offset=row_offset)
    exclude = None
    if excl_off is not None or excl_rows is not None:
        if excl_off is None or excl_rows is None:
            raise EbertError("cosine_topk: pass both excl_off and excl_rows, or neither")
        exclude = (excl_off.to(torch.int64).contiguous(), excl_rows.to(torch.int64).contiguous())
    return score_topk(catalog, k, queries=q, exclude=exclude)


@cosine_topk.register_fake
def _(q, cat, gnorm, inv, image, k, excl_off, excl_rows, row_offset):
    B = q.shape[0]
    return q.new_empty((B, k), dtype=torch.float64), q.new_empty((B, k), dtype=torch.int64)


@torch.library.custom_op("ebert::merge_topk", mutates_args=())
def merge_topk(scores: torch.Tensor, rows: torch.Tensor, k: int) -> Tuple[torch.Tensor,
                                                                          torch.Tensor]:
    """Merge R per-shard top-k lists ([R, B, k] f64 scores / i64 global rows, each sorted) into
    the global top-k (score desc, row asc)."""
    from .search import merge_topk as _merge
    return _merge(scores, rows, k)


@merge_topk.register_fake
def _(scores, rows, k):
    return (scores.new_empty((scores.shape[1], k), dtype=torch.float64),
            scores.new_empty((scores.shape[1], k), dtype=torch.int64))
