"""HBM-resident catalog: the GPU replacement of ``movies_collab_embeddings``.

Reference: ``src/backend/app/constants.py:55-56`` loads every movie vector from Chroma into a
float64 ``DataFrame(index=tmdb_id)`` at import time, and ``lib.py:51`` then re-normalises the
WHOLE catalog on every request (sklearn ``metrics/pairwise.py:1730-1734``). Here the catalog is
uploaded once, its guarded float64 row norms are computed once (``ebt_row_norms``), and the
MFMA screening image is built once:

* float16 / bfloat16 catalogs with d % 64 == 0 are screened NATIVELY: the matrix itself is the
  MFMA operand (no copy) and 1/||c|| is applied in the GEMM epilogue, so screening products are
  exact and only float32 accumulation error remains;
* float32 / float64 catalogs (and 16-bit ones with ragged d) get a float16 image of the
  NORMALISED rows, zero-padded to a multiple of 64 columns (unit round-off 2^-11, all values in
  [-1, 1]).

Either way the exact float64 scores are recomputed from the original matrix for the screened
candidates, so the image precision never reaches the results ("certified
screening").
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import DTYPE_CODE, EBT_BF16, EBT_F16, EbertError, call, ptr, require_cuda, stream_of

IMG_ALIGN = 64


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


class Catalog:
    """One (shard of a) catalog resident in HBM.

    Parameters
    ----------
    emb : CUDA tensor [n, d] of float32 / float64 / bfloat16 / float16, rows contiguous.
    ids : optional sequence of string ids (the DataFrame index of constants.py:56), one per row.
    row_offset : global row id of local row 0 when the catalog is row-sharded across ranks.
    n_global : total rows over all shards (defaults to n).
    """

    def __init__(self, emb: torch.Tensor, ids: Optional[Sequence[str]] = None,
                 row_offset: int = 0, n_global: Optional[int] = None) -> None:
        require_cuda(emb, "catalog embeddings")
        if emb.dim() != 2 or emb.shape[0] < 1 or emb.shape[1] < 1:
            raise EbertError(f"catalog must be a non-empty 2-D matrix, got {tuple(emb.shape)}")
        if emb.dtype not in DTYPE_CODE:
            raise EbertError(f"unsupported catalog dtype {emb.dtype}")
        if emb.stride(1) != 1:
            emb = emb.contiguous()
        self.data = emb
        self.device = emb.device
        self.n, self.d = int(emb.shape[0]), int(emb.shape[1])
        self.ld = int(emb.stride(0))
        self.dtype_code = DTYPE_CODE[emb.dtype]
        self.row_offset = int(row_offset)
        self.n_global = int(n_global) if n_global is not None else self.n
        self.d_pad = _round_up(self.d, IMG_ALIGN)
        st = stream_of(self.device)
        self.gnorm = torch.empty(self.n, dtype=torch.float64, device=self.device)
        self.inv32 = torch.empty(_round_up(self.n, 128), dtype=torch.float32, device=self.device)
        self.inv32[self.n:] = 1.0
        call("ebt_row_norms", ptr(emb), self.dtype_code, self.n, self.d, self.ld, ptr(self.gnorm),
             ptr(self.inv32), st)
        native_16 = emb.dtype in (torch.float16, torch.bfloat16)
        if native_16:
            self.img_dtype = EBT_F16 if emb.dtype == torch.float16 else EBT_BF16
            self.u_cat = 0.0
            self.cscale = self.inv32
            self.native = True
            if self.d % IMG_ALIGN == 0 and self.ld % IMG_ALIGN == 0 and emb.data_ptr() % 16 == 0:
                self.image = emb  # the matrix itself is the MFMA operand
                self.ld_img = self.ld
            else:
                self.ld_img = self.d_pad
                self.image = torch.empty((self.n, self.ld_img), dtype=emb.dtype, device=self.device)
                call("ebt_screen_image", ptr(emb), self.dtype_code, self.n, self.d, self.ld,
                     ptr(self.gnorm), 0, self.img_dtype, ptr(self.image), self.ld_img, st)
        else:
            self.img_dtype = EBT_F16
            self.u_cat = 2.0 ** -11
            self.cscale = None
            self.native = False
            self.ld_img = self.d_pad
            self.image = torch.empty((self.n, self.ld_img), dtype=torch.float16, device=self.device)
            call("ebt_screen_image", ptr(emb), self.dtype_code, self.n, self.d, self.ld,
                 ptr(self.gnorm), 1, self.img_dtype, ptr(self.image), self.ld_img, st)
        self.ids: Optional[List[str]] = list(ids) if ids is not None else None
        if self.ids is not None and len(self.ids) != self.n:
            raise EbertError(f"{len(self.ids)} ids for {self.n} rows")
        self._pos: Optional[Dict[str, int]] = None

    # ---- id helpers (the DataFrame index of constants.py:56) -----------------------------
    @classmethod
    def from_matrix(cls, ids: Optional[Sequence[str]], emb, device="cuda", **kw) -> "Catalog":
        if isinstance(emb, np.ndarray):
            emb = torch.from_numpy(np.ascontiguousarray(emb))
        return cls(emb.to(device), ids=ids, **kw)

    @property
    def index_pos(self) -> Dict[str, int]:
        if self.ids is None:
            raise EbertError("this catalog has no ids")
        if self._pos is None:
            self._pos = {t: i for i, t in enumerate(self.ids)}
        return self._pos

    def contains(self, tmdb_ids: Iterable[str]) -> List[bool]:
        pos = self.index_pos
        return [t in pos for t in tmdb_ids]

    def rows_of(self, tmdb_ids: Iterable[str]) -> List[int]:
        """Global row ids of the given string ids (KeyError for an unknown id)."""
        pos = self.index_pos
        return [pos[t] + self.row_offset for t in tmdb_ids]

    def id_of(self, global_row: int) -> str:
        return self.ids[global_row - self.row_offset]

    @property
    def img_torch_dtype(self) -> torch.dtype:
        return torch.float16 if self.img_dtype == EBT_F16 else torch.bfloat16

    def __repr__(self) -> str:
        return (f"Catalog(n={self.n}, d={self.d}, dtype={self.data.dtype}, row_offset="
                f"{self.row_offset}, image={'native' if self.native else 'f16-normalised'})")
