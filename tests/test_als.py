"""Implicit ALS: the float64 oracle against the objective it
minimises (CPU), and the HIP kernels (csrc/als.hip) against the oracle (GPU).

Spark (the reference's trainer, notebooks/create-embeddings.ipynb:1055) is not installed, so the
oracle restates its published computeFactors step and is pinned here by the implicit-feedback
objective itself (Hu, Koren & Volinsky; Spark's weighted lambda): parity with Spark's own
outputs is unpinned.
"""
import numpy as np
import pytest
import torch

from oracle import als as O


def _ratings(seed, n_users, n_items, per_user):
    rng = np.random.default_rng(seed)
    users, items, vals = [], [], []
    for u in range(n_users):
        k = int(rng.integers(1, per_user))
        its = rng.choice(n_items, k, replace=False)
        users += [u] * k
        items += its.tolist()
        vals += rng.choice([0.0, 0.5, 1.0, 2.5, 3.5, 4.0, 5.0, -1.0], k).tolist()
    return np.array(users), np.array(items), np.array(vals, dtype=np.float32)


def test_oracle_half_step_minimises_the_implicit_objective():
    """x_u from half_step zeroes the gradient of the DENSE implicit objective
    sum_i c_ui (p_ui - x.y_i)^2 + reg n_pos(u) |x|^2 over every item (unrated: c = 1, p = 0)."""
    n_users, n_items, rank, alpha, reg = 40, 60, 8, 1.0, 0.1
    users, items, vals = _ratings(1, n_users, n_items, 20)
    rng = np.random.default_rng(2)
    Y = rng.standard_normal((n_items, rank)).astype(np.float32)
    X = O.half_step(Y, *O.csr(users, items, vals, n_users), alpha, reg)
    Y64 = Y.astype(np.float64)
    for u in range(n_users):
        c = np.ones(n_items)
        p = np.zeros(n_items)
        m = users == u
        c[items[m]] = 1.0 + alpha * np.abs(vals[m])
        p[items[m]] = (vals[m] > 0).astype(np.float64)
        x = X[u].astype(np.float64)
        grad = -2 * ((c * (p - Y64 @ x))[:, None] * Y64).sum(0) + 2 * reg * (vals[m] > 0).sum() * x
        assert np.abs(grad).max() < 1e-4 * max(1.0, np.abs(x).max()) * n_items


@pytest.mark.gpu
def test_gpu_gram_and_half_step(cuda_device):
    from robot_ebert_amd import als
    n_users, n_items, rank = 300, 500, 32
    users, items, vals = _ratings(3, n_users, n_items, 80)
    rng = np.random.default_rng(4)
    Y = rng.standard_normal((n_items, rank)).astype(np.float32)
    Yt = torch.from_numpy(Y).to(cuda_device)
    G = als.gram(Yt).cpu().numpy()
    assert np.allclose(G, Y.astype(np.float64).T @ Y.astype(np.float64), rtol=1e-12, atol=1e-9)
    R = als.Ratings(users, items, vals, n_users, n_items, cuda_device)
    X = als.half_step(Yt, R.by_user, 1.0, 0.1).cpu().numpy()
    want = O.half_step(Y, *O.csr(users, items, vals, n_users), 1.0, 0.1)
    np.testing.assert_allclose(X, want, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_gpu_train_matches_oracle(cuda_device):
    """Three ALS iterations (rank 32, reg 0.1, alpha 1) from the same starting factors."""
    from robot_ebert_amd import als
    n_users, n_items, rank = 200, 400, 32
    users, items, vals = _ratings(5, n_users, n_items, 60)
    U0 = als.init_factors(n_users, rank, 7, "cpu").numpy()
    V0 = als.init_factors(n_items, rank, 8, "cpu").numpy()
    R = als.Ratings(users, items, vals, n_users, n_items, cuda_device)
    U, V = als.train(R, rank=rank, iters=3, U0=torch.from_numpy(U0), V0=torch.from_numpy(V0))
    Uw, Vw = O.train(users, items, vals, n_users, n_items, U0, V0, 3)
    np.testing.assert_allclose(U.cpu().numpy(), Uw, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(V.cpu().numpy(), Vw, rtol=1e-4, atol=1e-5)
    # an item without ratings gets the zero factor (b = 0), as Spark would never emit it
    empty = np.setdiff1d(np.arange(n_items), items)
    if empty.size:
        assert float(V[torch.from_numpy(empty)].abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("rank", [5, 48])
def test_gpu_half_step_other_ranks(cuda_device, rank):
    """The padded register blocks: a rank below the 2 x 2 tiling and one on the 4 x 4 kernel."""
    from robot_ebert_amd import als
    n_users, n_items = 120, 200
    users, items, vals = _ratings(9, n_users, n_items, 50)
    rng = np.random.default_rng(10)
    Y = rng.standard_normal((n_items, rank)).astype(np.float32)
    R = als.Ratings(users, items, vals, n_users, n_items, cuda_device)
    X = als.half_step(torch.from_numpy(Y).to(cuda_device), R.by_user, 1.0, 0.1).cpu().numpy()
    want = O.half_step(Y, *O.csr(users, items, vals, n_users), 1.0, 0.1)
    np.testing.assert_allclose(X, want, rtol=2e-5, atol=2e-6)
