"""ctypes binding of libebert.so (the C ABI declared in include/ebert.h).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C robot_ebert_amd/csrc``).
There is no fallback: if the shared object is missing or fails to load, every entry point
raises ``EbertError`` -- the product path never silently computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EBERT_LIB", os.path.join(_HERE, "libebert.so"))

EBT_F32, EBT_BF16, EBT_F16, EBT_F64 = 0, 1, 2, 3
DTYPE_CODE = {torch.float32: EBT_F32, torch.bfloat16: EBT_BF16, torch.float16: EBT_F16,
              torch.float64: EBT_F64}
STAGES = {"gemm": 0, "mask": 1, "select": 2, "merge_select": 3, "rescore": 4, "gemm_filter": 5,
          "prep": 6, "shard_merge": 7, "collective_wait": 8, "small": 9}
EBT_FLAG_NO_FUSE = 1
EBT_FLAG_EXACT = 2
EBT_FLAG_THETA = 4
EBT_FLAG_LIKED_CHECKED = 8   # ebert.h: the liked CSR was checked on the host (no read-back)
EBT_FILTER_SLOTS_MAX = 128


class EbertError(RuntimeError):
    """A libebert call failed (or the library could not be loaded)."""


_VP, _I32, _I64, _SZ, _F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
_INT = ctypes.c_int

class EbtCatalog(ctypes.Structure):
    """include/ebert.h `ebt_catalog` (filled by ebt_catalog_init)."""
    _fields_ = [("data", _VP), ("dtype", _I32), ("d", _I32), ("n", _I64), ("ld", _I64),
                ("row_offset", _I64), ("gnorm64", _VP), ("inv32", _VP), ("image", _VP),
                ("cscale", _VP), ("img_dtype", _I32), ("ld_img", _I32), ("d_pad", _I32),
                ("native", _I32), ("u_cat", _F32)]


class EbtOptions(ctypes.Structure):
    """include/ebert.h `ebt_options` (zero fields = defaults)."""
    _fields_ = [("kprime", _I32), ("flags", _I32), ("chunk_rows", _I64)]


class EbtPending(ctypes.Structure):
    """include/ebert.h `ebt_pending`: a submitted batch (ebt_cosine_topk_submit / _finish)."""
    _fields_ = [("cat", _VP), ("opt", EbtOptions), ("B", _I64), ("B_pad", _I64),
                ("chunk", _I64), ("k", _I32), ("k_eff", _I32), ("kprime", _I32),
                ("flags", _I32), ("excl_off", _VP), ("excl_rows", _VP), ("ws", _VP),
                ("ws_bytes", _SZ), ("out_scores", _VP), ("out_rows", _VP), ("cert_host", _VP),
                ("event", _VP), ("timer", _VP), ("stream", _VP)]


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _VP, _SZ, _VP)


ALLREDUCE_F64_FN = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _SZ, _VP)


class EbtComm(ctypes.Structure):
    """include/ebert.h `ebt_comm`: the caller's all-gather (and optional float64 all-reduce)
    for ebt_cosine_topk_sharded."""
    _fields_ = [("rank", _I32), ("world", _I32), ("n_global", _I64),
                ("all_gather", ALLGATHER_FN), ("ctx", _VP),
                ("all_reduce_f64", ALLREDUCE_F64_FN)]


class EbtShardedPending(ctypes.Structure):
    """include/ebert.h `ebt_sharded_pending`: a row-sharded batch in flight
    (ebt_cosine_topk_sharded_submit / _finish / _wait)."""
    _fields_ = [("local", EbtPending), ("comm", EbtComm), ("out_scores", _VP),
                ("out_rows", _VP), ("host", _VP), ("event", _VP), ("stage", _I32)]


_PCAT, _POPT, _PPEND = (ctypes.POINTER(EbtCatalog), ctypes.POINTER(EbtOptions),
                        ctypes.POINTER(EbtPending))
_PCOMM = ctypes.POINTER(EbtComm)
_PSPEND = ctypes.POINTER(EbtShardedPending)

_SIGNATURES = {
    "ebt_catalog_state_bytes": ([_VP, _INT, _I64, _I32, _I64], _SZ),
    "ebt_catalog_init": ([_PCAT, _VP, _INT, _I64, _I32, _I64, _I64, _VP, _SZ, _VP], _INT),
    "ebt_workspace_bytes": ([_PCAT, _I64, _I32, _POPT], _SZ),
    "ebt_cosine_topk": ([_PCAT, _VP, _INT, _I64, _I64, _VP, _VP, _I32, _VP, _VP, _POPT, _VP, _SZ,
                         _VP, _VP, _VP, _VP], _INT),
    "ebt_cosine_topk_submit": ([_PCAT, _VP, _INT, _I64, _I64, _VP, _VP, _I32, _VP, _VP, _POPT,
                                _VP, _SZ, _VP, _VP, _VP, _PPEND, _VP, _VP], _INT),
    "ebt_cosine_topk_finish": ([_PPEND], _INT),
    "ebt_sharded_workspace_bytes": ([_PCAT, _PCOMM, _I64, _I32, _POPT], _SZ),
    "ebt_cosine_topk_sharded": ([_PCAT, _PCOMM, _VP, _INT, _I64, _I64, _VP, _VP, _I32, _VP, _VP,
                                 _POPT, _VP, _SZ, _VP, _VP, _VP, _VP], _INT),
    "ebt_cosine_topk_sharded_submit": ([_PCAT, _PCOMM, _VP, _INT, _I64, _I64, _VP, _VP, _I32,
                                        _VP, _VP, _POPT, _VP, _SZ, _VP, _VP, _VP, _PSPEND, _VP,
                                        _VP], _INT),
    "ebt_cosine_topk_sharded_finish": ([_PSPEND], _INT),
    "ebt_cosine_topk_sharded_wait": ([_PSPEND], _INT),
    "ebt_rccl_unique_id": ([_VP, _SZ], _INT),
    "ebt_rccl_comm_init": ([_VP, _I32, _I32, ctypes.POINTER(_VP)], _INT),
    "ebt_rccl_comm_destroy": ([_VP], _INT),
    "ebt_rccl_all_gather": ([_VP, _VP, _VP, _SZ, _VP], _INT),
    "ebt_rccl_all_reduce_f64": ([_VP, _VP, _SZ, _VP], _INT),
    "ebt_shard_list_width": ([_I32, _I32], _I64),
    "ebt_shard_sample_tiles": ([_I64, _I32, _I64], _I64),
    "ebt_shard_pack_cap": ([_I64, _I32, _I32, _I64], _I64),
    "ebt_shard_pack_bytes": ([_I64, _I64], _SZ),
    "ebt_shard_pack": ([_VP, _VP, _I64, _I32, _VP, _I64, _VP, _VP], _INT),
    "ebt_merge_packed": ([_VP, _I32, _I64, _I32, _I64, _VP, _VP, _VP, _VP], _INT),
    "ebt_floor_pack": ([_VP, _I64, _I64, _I32, _I32, _VP, _VP, _VP], _INT),
    "ebt_version": ([], _INT),
    "ebt_last_error": ([], ctypes.c_char_p),
    "ebt_row_norms": ([_VP, _INT, _I64, _I32, _I64, _VP, _VP, _VP], _INT),
    "ebt_screen_image": ([_VP, _INT, _I64, _I32, _I64, _VP, _INT, _INT, _VP, _I32, _VP], _INT),
    "ebt_query_dense": ([_VP, _INT, _I64, _I32, _I64, _VP, _VP], _INT),
    "ebt_query_liked_sum": ([_VP, _INT, _I32, _I64, _VP, _I64, _VP, _VP, _VP, _VP], _INT),
    "ebt_scale_rows_f64": ([_VP, _I64, _I32, _VP, _VP], _INT),
    "ebt_query_prep": ([_VP, _INT, _I64, _I64, _I32, _I64, _INT, _INT, _F32, _VP, _VP, _I32, _VP,
                        _VP, _VP], _INT),
    "ebt_query_image": ([_VP, _I64, _I64, _I32, _INT, _VP, _I64, _INT, _F32, _VP, _I32, _VP, _VP,
                         _VP], _INT),
    "ebt_screen_scores": ([_VP, _I64, _VP, _I64, _I32, _I32, _INT, _VP, _VP, _VP, _I64, _VP],
                          _INT),
    "ebt_screen_filter": ([_VP, _I64, _VP, _I64, _I32, _I32, _INT, _VP, _VP, _VP, _VP, _I64, _I32,
                           _VP, _I64, _VP, _I64, _VP], _INT),
    "ebt_filter_group_rows": ([_I64], _I64),
    "ebt_merge_block_max_groups": ([_I32], _I64),
    "ebt_cosine_topk_spec_lead": ([_I64, _I64, _I64, _I32, _INT], _I64),
    "ebt_spec_lead": ([_INT], _INT),
    "ebt_filter_split": ([_I64], _I64),
    "ebt_cosine_screen": ([_VP, _VP, _VP, _VP, _I64, _I64, _VP, _INT, _I64, _VP, _VP, _VP, _INT,
                           _I32, _I64, _I32, _I32, _I64, _VP, _VP, _I32, _I32, _I64, _INT, _VP,
                           ctypes.c_size_t, _VP, _VP, _VP, _VP, _VP, _VP], _INT),
    "ebt_cosine_screen_at": ([_VP, _VP, _VP, _VP, _I64, _I64, _VP, _INT, _I64, _VP, _VP, _VP,
                              _INT, _I32, _I64, _I32, _I32, _I64, _VP, _VP, _I32, _I32, _I64,
                              _INT, _VP, ctypes.c_size_t, _VP, _VP, _VP, _VP, _VP,
                              ctypes.c_double, _VP, _VP], _INT),
    "ebt_cosine_sample": ([_VP, _VP, _I64, _VP, _VP, _INT, _I32, _I64, _I32, _I64, _I64, _VP,
                           _I64, _VP, _VP], _INT),
    "ebt_cosine_sample_lead": ([_VP, _VP, _I64, _VP, _VP, _INT, _I32, _I64, _I32, _I64, _I64,
                                _VP, _I64, _I64, _VP, _I64, _VP, _VP], _INT),
    "ebt_cosine_screen_at_lead": ([_VP, _VP, _VP, _VP, _I64, _I64, _VP, _INT, _I64, _VP, _VP,
                                   _VP, _INT, _I32, _I64, _I32, _I32, _I64, _VP, _VP, _I32,
                                   _I32, _I64, _INT, _VP, ctypes.c_size_t, _VP, _VP, _VP, _VP,
                                   _VP, ctypes.c_double, _I64, _VP, _I64, _VP, _VP], _INT),
    "ebt_pool_kth": ([_VP, _I64, _I64, _I64, _I32, _I32, _VP, _VP], _INT),
    "ebt_union_floor": ([_VP, _I32, _I64, _I32, _I32, _VP, _VP], _INT),
    "ebt_certify_cut": ([_VP, _VP, _VP, _VP, _VP, _I64, _VP], _INT),
    "ebt_rescore_owned": ([_VP, _I64, _I32, _VP, _INT, _I64, _VP, _I64, _I64, _VP, _VP, _I32,
                           _I32, _VP, _VP, _VP], _INT),
    "ebt_finalize_topk": ([_VP, _VP, _VP, _I64, _I32, _I32, _I64, _VP, _VP, _VP, _VP, _VP, _VP],
                          _INT),
    "ebt_merge_hits": ([_VP, _VP, _I64, _I32, _I32, _VP, _I64, _I32, _VP, _I64, _I64, _I64, _VP, _VP, _VP,
                        _VP], _INT),
    "ebt_mask_excluded": ([_VP, _I64, _I64, _I64, _I64, _VP, _VP, _VP], _INT),
    "ebt_select_topk": ([_VP, _VP, _I64, _I64, _I64, _I64, _I32, _I32, _VP, _VP, _I64, _VP],
                        _INT),
    "ebt_rescore": ([_VP, _I64, _I32, _VP, _INT, _I64, _VP, _I64, _VP, _VP, _I32, _I32, _I64, _VP,
                     _VP, _VP, _VP, _VP, _VP, _VP], _INT),
    "ebt_rescore_form": ([_INT], _INT),
    "ebt_wave_sum_check": ([_VP, _I64, _VP, _VP, _VP], _INT),
    "ebt_sort_exclusions_bytes": ([_I64, _I64], _SZ),
    "ebt_sort_exclusions": ([_VP, _VP, _VP, _I64, _I64, _VP, _SZ, _VP], _INT),
    "ebt_merge_topk": ([_VP, _VP, _I32, _I64, _I32, _VP, _VP, _VP], _INT),
    "ebt_screen_exact": ([_VP, _I64, _I32, _VP, _INT, _I64, _VP, _I64, _VP, _I64, _VP], _INT),
    "ebt_cosine_topk_workspace": ([_I64, _I64, _I64, _I32, _I64, _INT], _SZ),
    "ebt_cosine_topk_plan": ([_I64, _I64, _I64, _I32, _I64, _INT, ctypes.POINTER(_I64),
                              ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                              ctypes.POINTER(ctypes.c_int32)], _INT),
    "ebt_cosine_topk_spec_plan": ([_I64, _I64, _I64, _I32, _INT, ctypes.POINTER(_I64),
                                   ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int32),
                                   ctypes.POINTER(ctypes.c_double)], _INT),
    "ebt_cosine_topk_prepared": ([_VP, _VP, _VP, _VP, _I64, _I64, _VP, _INT, _I64, _VP, _VP, _VP, _INT,
                         _I32, _I64, _I32, _I32, _I64, _VP, _VP, _I32, _I32, _I64, _INT, _VP, _SZ,
                         _VP, _VP, _VP, _VP, _VP], _INT),
    "ebt_als_gram": ([_VP, _I64, _I32, _VP, _VP], _INT),
    "ebt_als_solve": ([_VP, _VP, _I32, _I64, _VP, _VP, _VP, _F32, _F32, _VP, _VP], _INT),
    "ebt_timer_create": ([], _VP),
    "ebt_timer_destroy": ([_VP], None),
    "ebt_timer_reset": ([_VP], _INT),
    "ebt_timer_set_mask": ([_VP, ctypes.c_uint32], _INT),
    "ebt_timer_query": ([_VP, _INT, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64)], _INT),
    "ebt_timer_begin": ([_VP, _INT, _VP], _INT),
    "ebt_timer_end": ([_VP, _INT, _VP], _INT),
    "ebt_timer_count_rows": ([_VP, _INT], _INT),
    "ebt_timer_rows": ([_VP, ctypes.POINTER(_I64)], _INT),
}

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Load libebert.so once; raise EbertError if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise EbertError(
                    f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                    "g.build()'` (make -C robot_ebert_amd/csrc)")
            try:
                lib = ctypes.CDLL(LIB_PATH)
            except OSError as e:
                raise EbertError(f"cannot load {LIB_PATH}: {e}") from e
            for name, (args, res) in _SIGNATURES.items():
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = res
            _lib = lib
    return _lib


def call(name: str, *args) -> int:
    """Call an ``int``-returning entry point and raise EbertError on a negative status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.ebt_last_error().decode(errors="replace")
        raise EbertError(f"{name} failed with status {rc}: {msg}")
    return rc


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_of(device: torch.device) -> int:
    """The current torch (HIP) stream of `device`: every libebert call enqueues on it."""
    return torch.cuda.current_stream(device).cuda_stream


def require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise EbertError(f"{what} must be a CUDA (HIP) tensor; libebert has no CPU path")


class Timer:
    """Per-stage GPU time collected with hipEvents on the launch stream (ebt_timer_*)."""

    def __init__(self) -> None:
        self._h = load().ebt_timer_create()
        if not self._h:
            raise EbertError("ebt_timer_create failed")

    def reset(self) -> None:
        call("ebt_timer_reset", self._h)

    def only(self, *stages: str) -> None:
        """Record only these stages from now on (all of them when none are given)."""
        mask = 0xffffffff if not stages else sum(1 << STAGES[s] for s in stages)
        call("ebt_timer_set_mask", self._h, mask)

    def query(self, stage: str):
        tot = ctypes.c_double(0.0)
        n = ctypes.c_int64(0)
        call("ebt_timer_query", self._h, STAGES[stage], ctypes.byref(tot), ctypes.byref(n))
        return tot.value, n.value

    def count_rows(self, on: bool = True) -> None:
        """Count the candidate rows the rescore gathers (top-K roofline bytes; ebt_timer_rows)."""
        call("ebt_timer_count_rows", self._h, 1 if on else 0)

    def rows(self) -> int:
        """Candidate rows gathered by the recorded rescores since the last reset."""
        n = ctypes.c_int64(0)
        call("ebt_timer_rows", self._h, ctypes.byref(n))
        return n.value

    def region(self, stage: str, device=None):
        """Context manager: the work enqueued on the current stream inside the block is one
        record of `stage` (ebt_timer_begin / ebt_timer_end)."""
        return _Region(self, STAGES[stage], device)

    @property
    def handle(self) -> int:
        return self._h

    def __del__(self):
        try:
            if self._h and _lib is not None:
                _lib.ebt_timer_destroy(self._h)
        except Exception:
            pass
        self._h = None


class _Region:
    def __init__(self, timer: "Timer", stage: int, device) -> None:
        self.t, self.stage, self.device = timer, stage, device

    def __enter__(self):
        call("ebt_timer_begin", self.t.handle, self.stage, stream_of(self.device))
        return self

    def __exit__(self, *exc):
        call("ebt_timer_end", self.t.handle, self.stage, stream_of(self.device))
        return False


def region(timer: Optional["Timer"], stage: str, device=None):
    """timer.region(stage) or a no-op when timer is None."""
    import contextlib
    return timer.region(stage, device) if timer is not None else contextlib.nullcontext()
