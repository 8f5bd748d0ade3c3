"""CPU: the route wiring of robot_ebert_amd.api (api/users.py:150-155) with the scoring call
stubbed -- path, query parameter default, response JSON shape, and an uncaught ValueError
answered with HTTP 500 as in the reference app. The GPU test
test_gpu_parity.py::test_route_recommendations_matches_reference runs it on the real path."""
import datetime

from fastapi.testclient import TestClient

from robot_ebert_amd import api, lib
from robot_ebert_amd.models import Movie, Recommendation


def _movie(t):
    return Movie(tmdb_id=t, tmdb_homepage="", title=t, language="en",
                 release_date=datetime.date(2000, 1, 1), runtime=90, director="d", actors=None,
                 genres=None, keywords=None, overview="", budget=0, revenue=0, popularity=1.0,
                 vote_average=0.0, vote_count=0)


def test_route_wiring(monkeypatch):
    calls = []

    def fake(user_id, k=10):
        calls.append((user_id, k))
        if user_id == "nolike":
            raise ValueError("Found array with 0 sample(s)")
        if user_id == "new":
            return []
        return [Recommendation(movie=_movie(str(i)), score=1.0 - i / 10) for i in range(k)]
    monkeypatch.setattr(lib, "get_user_recs", fake)
    c = TestClient(api.app(), raise_server_exceptions=False)
    r = c.get("/users/u1/recommendations/")
    assert r.status_code == 200 and len(r.json()) == 10 and calls[-1] == ("u1", 10)
    r = c.get("/users/u1/recommendations/", params={"k": 3})
    assert [x["movie"]["tmdb_id"] for x in r.json()] == ["0", "1", "2"]
    assert [x["score"] for x in r.json()] == [1.0, 0.9, 0.8]
    assert c.get("/users/new/recommendations/").json() == []
    assert c.get("/users/nolike/recommendations/").status_code == 500
    assert c.get("/users/u1/recommendations/", params={"k": "x"}).status_code == 422
