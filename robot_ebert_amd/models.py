"""Response types of the recommend path (mirror of src/shared/models.py:33-49,73-75).

Only the types the hot path returns are mirrored; the reference's module also imports
llama_index message types for its chat endpoints, which are out of scope here.
"""
from __future__ import annotations

from datetime import date
from typing import List, Optional

from pydantic import BaseModel


class Movie(BaseModel):  # shared/models.py:33-49
    tmdb_id: str
    tmdb_homepage: str
    title: str
    language: str
    release_date: date
    runtime: int
    director: str
    actors: Optional[List[str]]
    genres: Optional[List[str]]
    keywords: Optional[List[str]]
    overview: str
    budget: int
    revenue: int
    popularity: float
    vote_average: float
    vote_count: int


class Recommendation(BaseModel):  # shared/models.py:73-75
    movie: Movie
    score: float
