"""robot_ebert_amd -- MI355X-native embedding-similarity retrieval for robot-ebert's recommend path.

The hot path (query x catalog cosine + top-k, reference src/backend/app/lib.py:51-55) runs in
hand-written HIP kernels for gfx950 behind the C ABI of include/ebert.h (libebert.so, loaded by
ctypes). Python keeps the reference's call surface: ``lib.get_user_recs`` and friends.
"""
from ._lib import EbertError, Timer, load  # noqa: F401
from .catalog import Catalog  # noqa: F401
from .search import (merge_topk, prepare_queries, rescore_rows, score_topk,  # noqa: F401
                     score_topk_finish, score_topk_submit)
from . import ops  # noqa: F401,E402  (registers torch.ops.ebert.*)

__version__ = "0.1.0"
