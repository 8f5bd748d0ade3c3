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

import ctypes
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import DTYPE_CODE, EBT_BF16, EBT_F16, EbertError, call, ptr, require_cuda, stream_of  # noqa: F401

IMG_ALIGN = 64


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def _al(v: int) -> int:
    """ebt_catalog_init's state-buffer alignment (256 bytes)."""
    return _round_up(v, 256)


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
        # the C ABI's catalog (ebt_catalog_init): guarded float64 norms, float32 inverse norms
        # and the screening image in one device state buffer owned here
        lib = _lib.load()
        need = lib.ebt_catalog_state_bytes(ptr(emb), self.dtype_code, self.n, self.d, self.ld)
        if need == 0:
            raise EbertError(f"bad catalog shape {tuple(emb.shape)} (ld {self.ld})")
        self.state = torch.empty(need, dtype=torch.uint8, device=self.device)
        self.cstruct = _lib.EbtCatalog()
        call("ebt_catalog_init", ctypes.byref(self.cstruct), ptr(emb), self.dtype_code, self.n,
             self.d, self.ld, self.row_offset, ptr(self.state), need, stream_of(self.device))
        c = self.cstruct
        off_inv = _al(self.n * 8)
        n128 = _round_up(self.n, 128)
        off_img = off_inv + _al(n128 * 4)
        self.gnorm = self.state[:self.n * 8].view(torch.float64)
        self.inv32 = self.state[off_inv:off_inv + n128 * 4].view(torch.float32)
        self.img_dtype = int(c.img_dtype)
        self.ld_img = int(c.ld_img)
        self.native = bool(c.native)
        self.u_cat = float(c.u_cat)
        self.cscale = self.inv32 if self.native else None
        if c.image == emb.data_ptr():
            self.image = emb  # the matrix itself is the MFMA operand
        else:
            self.image = self.state[off_img:off_img + self.n * self.ld_img * 2].view(
                self.img_torch_dtype).view(self.n, self.ld_img)
        self.ids: Optional[List[str]] = list(ids) if ids is not None else None
        if self.ids is not None and len(self.ids) != self.n:
            raise EbertError(f"{len(self.ids)} ids for {self.n} rows")
        self._pos: Optional[Dict[str, int]] = None

    # ---- constructors ---------------------------------------------------------------------
    @classmethod
    def from_matrix(cls, ids: Optional[Sequence[str]], emb, device="cuda", shard: bool = False,
                    **kw) -> "Catalog":
        """SURVEY §8b's ``Catalog.from_matrix(ids, emb, shard)``: upload a host or device matrix.
        With ``shard=True`` (an initialised torch.distributed group) this rank keeps only its
        row range ``shard_range(n, rank, world)`` (ids sliced alike); rows stay GLOBAL ids."""
        if isinstance(emb, np.ndarray):
            emb = torch.from_numpy(np.ascontiguousarray(emb))
        if shard:
            import torch.distributed as dist
            from .distributed import shard_range
            if not (dist.is_available() and dist.is_initialized()):
                raise EbertError("shard=True needs an initialised torch.distributed process group")
            n = int(emb.shape[0])
            a, b = shard_range(n, dist.get_rank(), dist.get_world_size())
            emb = emb[a:b]
            ids = list(ids)[a:b] if ids is not None else None
            kw = dict(kw, row_offset=a, n_global=n)
        return cls(emb.to(device), ids=ids, **kw)

    @classmethod
    def from_parts(cls, emb: torch.Tensor, gnorm: torch.Tensor, inv32: torch.Tensor,
                   image: torch.Tensor, row_offset: int = 0,
                   n_global: Optional[int] = None) -> "Catalog":
        """A catalog view over tensors already built by ``row_norms`` / ``screen_image`` (the
        torch ops of ``ops.py``): nothing is recomputed. ``image`` is the f16 normalised image,
        or the matrix itself for a native f16/bf16 catalog with d % 64 == 0."""
        for t, what in ((emb, "catalog"), (gnorm, "gnorm"), (inv32, "inv"), (image, "image")):
            require_cuda(t, what)
        self = cls.__new__(cls)
        self.data = emb if emb.stride(1) == 1 else emb.contiguous()
        self.device = emb.device
        self.n, self.d = int(emb.shape[0]), int(emb.shape[1])
        self.ld = int(self.data.stride(0))
        self.dtype_code = DTYPE_CODE[emb.dtype]
        self.row_offset = int(row_offset)
        self.n_global = int(n_global) if n_global is not None else self.n
        self.d_pad = _round_up(self.d, IMG_ALIGN)
        if gnorm.dtype != torch.float64 or gnorm.numel() < self.n:
            raise EbertError("gnorm must be float64 [n]")
        if inv32.dtype != torch.float32 or inv32.numel() < _round_up(self.n, 128):
            raise EbertError("inv must be float32 [round_up(n, 128)]")
        self.gnorm, self.inv32 = gnorm, inv32
        native_16 = emb.dtype in (torch.float16, torch.bfloat16)
        if image.dtype not in (torch.float16, torch.bfloat16) or image.shape[0] != self.n or \
                image.stride(1) != 1 or image.stride(0) % IMG_ALIGN or image.shape[1] < self.d_pad:
            raise EbertError("image must be a 16-bit [n, >= round_up(d, 64)] matrix, "
                             "row stride a multiple of 64")
        self.image, self.ld_img = image, int(image.stride(0))
        self.img_dtype = EBT_F16 if image.dtype == torch.float16 else EBT_BF16
        self.native = native_16  # the image holds the raw rows, scaled by inv in the epilogue
        self.u_cat = 0.0 if native_16 else 2.0 ** -11
        self.cscale = self.inv32 if native_16 else None
        self.ids, self._pos = None, None
        self.state = None
        self.cstruct = _lib.EbtCatalog(
            data=ptr(self.data), dtype=self.dtype_code, d=self.d, n=self.n, ld=self.ld,
            row_offset=self.row_offset, gnorm64=ptr(gnorm), inv32=ptr(inv32), image=ptr(image),
            cscale=ptr(self.cscale), img_dtype=self.img_dtype, ld_img=self.ld_img,
            d_pad=self.d_pad, native=1 if native_16 else 0, u_cat=self.u_cat)
        return self

    # ---- id helpers (the DataFrame index of constants.py:56) -----------------------------

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
