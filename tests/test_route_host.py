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


def test_user_request_lists_match_dataframe_path():
    """lib._user_request's plain-Python filtering (lib.py:43-48) gives the lists
    lib.user_query_lists builds from the pandas DataFrame: catalog movies only, liked rows in
    rating order of the query result, rated ids in first-seen order, the sklearn error text for
    a user without a liked catalog movie, None for a user without ratings."""
    import pandas as pd
    import pytest
    from sqlalchemy import create_engine, insert
    from sqlalchemy.pool import StaticPool
    from robot_ebert_amd import tables

    class Cat:   # the id helpers of robot_ebert_amd.catalog.Catalog, no device
        d, row_offset = 8, 100

        def __init__(self, ids):
            self.ids = ids
            self.index_pos = {t: i for i, t in enumerate(ids)}

        def contains(self, ts):
            return [t in self.index_pos for t in ts]

        def rows_of(self, ts):
            return [self.index_pos[t] + self.row_offset for t in ts]
    cat = Cat([str(1000 + i) for i in range(50)])
    eng = create_engine("sqlite://", connect_args={"check_same_thread": False},
                        poolclass=StaticPool)
    tables.ratings.create(eng)
    rng = __import__("numpy").random.default_rng(4)
    users = {}
    with eng.begin() as cnx:
        for u in range(30):
            ids = rng.choice(70, 12, replace=False)   # ids >= 1050 are not in the catalog
            rts = rng.choice([0.5, 2.0, 3.4, 3.5, 4.0, 5.0], 12)
            if u == 7:
                rts[:] = 1.0                          # no liked movie
            users[f"u{u}"] = list(zip([str(1000 + int(i)) for i in ids], rts.tolist()))
            for t, rt in users[f"u{u}"]:
                cnx.execute(insert(tables.ratings).values(user_id=f"u{u}", tmdb_id=t, rating=rt))
    lib.configure(engine=eng, catalog=cat)
    for uid in users:
        with eng.begin() as cnx:
            rows = cnx.execute(tables.ratings.select().where(tables.ratings.c.user_id == uid)).all()
        df = pd.DataFrame(rows)
        df = df[df["tmdb_id"].isin(cat.index_pos.keys())]
        want = lib.user_query_lists(df, cat)
        if not want[0]:
            with pytest.raises(ValueError, match="Found array with 0 sample"):
                lib._user_request(uid)
            continue
        assert lib._user_request(uid) == (list(want[0]), list(want[1])), uid
    assert lib._user_request("nobody") is None
