"""The recommend route, unchanged, over the GPU drop-in.

Mirrors /root/reference/src/backend/app/api/users.py:150-155 -- same path, same query
parameter, same response model, same behaviour on errors: ``get_user_recs`` raising (sklearn's
ValueError for a user without liked movies, lib.py:51) is not caught, so the server answers
HTTP 500 exactly as the reference's app does. The only difference is the import: the handler
calls ``robot_ebert_amd.lib.get_user_recs`` (HBM-resident catalog, HIP scoring) instead of
``backend.app.lib.get_user_recs`` (sklearn + pandas). ``app()`` assembles a FastAPI app the
way /root/reference/src/backend/app/main.py:11-12 does (users router, tag "Users"); the
reference's other routers (movies, search, login) are out of scope.
"""
from __future__ import annotations

from typing import List

from fastapi import APIRouter, FastAPI

from . import lib
from .models import Recommendation

router = APIRouter()
# a batcher.RecBatcher installed by app(batcher=...): the handler's scoring step is then
# coalesced with the other worker threads' requests; None = one call per request
_batcher = None


@router.get("/users/{user_id}/recommendations/")
def get_user_recommendations(user_id: str, k: int = 10) -> List[Recommendation]:
    """get unconditional movie recommendations for an existing user by ID"""
    if _batcher is not None:
        return lib.get_user_recs_batched(_batcher, user_id=user_id, k=k)
    user_recommendations = lib.get_user_recs(user_id=user_id, k=k)
    return user_recommendations


def app(batcher=None) -> FastAPI:
    """FastAPI app with the users router (main.py:11-12); configure ``lib`` first. With a
    ``batcher.RecBatcher`` over ``lib.movies_collab_catalog`` the route's requests share GPU
    batches (same answers, same errors)."""
    global _batcher
    _batcher = batcher
    a = FastAPI()
    a.include_router(router, tags=["Users"])
    return a
