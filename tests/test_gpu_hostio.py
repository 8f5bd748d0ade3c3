"""GPU: the overlapped host boundary (robot_ebert_amd/hostio.py) returns exactly what the
resident path returns: hostio.run_pipelined over host query batches (H2D / D2H on the copy
stream, batches in flight), including a batch with k beyond the catalog (the C entry's padding
runs in its finish: the D2H must wait for it) and the liked-CSR path through a HostStager with
EBT_FLAG_LIKED_CHECKED (no read-back in the submit)."""
import numpy as np
import pytest
import torch

from oracle import restatement as R

pytestmark = pytest.mark.gpu


def test_run_pipelined_equals_resident(cuda_device):
    import robot_ebert_amd as ebt
    from robot_ebert_amd.hostio import HostStager, run_pipelined
    n, d, B, k = 30_000, 96, 300, 20
    g = torch.Generator().manual_seed(4)
    c = torch.randn((n, d), generator=g)
    cat = ebt.Catalog(c.to(cuda_device))
    qs = [torch.randn((B, d), generator=g) for _ in range(5)]
    st = HostStager(cuda_device)
    want = [ebt.score_topk(cat, k, queries=q.to(cuda_device)) for q in qs]
    got = [h.result() for h in run_pipelined(
        st, [q.pin_memory() for q in qs],
        lambda qd: ebt.score_topk_submit(cat, k, queries=qd),
        ebt.score_topk_finish)]
    for (ws, wr), (s, r) in zip(want, got):
        assert np.array_equal(r, wr.cpu().numpy())
        assert np.array_equal(s, ws.cpu().numpy())
    # k past the catalog: padded in the finish (a fresh event for the D2H)
    small = ebt.Catalog(c[:50].to(cuda_device))
    got2 = [h.result() for h in run_pipelined(
        st, [q.pin_memory() for q in qs[:3]],
        lambda qd: ebt.score_topk_submit(small, 64, queries=qd), ebt.score_topk_finish)]
    for q, (s, r) in zip(qs[:3], got2):
        s_ref, r_ref = R.cosine_topk(q.double().numpy(), c[:50].double().numpy(), 64)
        assert np.array_equal(r, r_ref)
        assert np.all(np.isnan(s[:, 50:])) and np.all(r[:, 50:] == -1)


def test_liked_checked_through_stager(cuda_device):
    import robot_ebert_amd as ebt
    from robot_ebert_amd.hostio import HostStager
    from robot_ebert_amd.search import csr_from_lists
    n, d, k = 20_000, 64, 15
    rng = np.random.default_rng(6)
    x = rng.standard_normal((n, d))
    cat = ebt.Catalog(torch.tensor(x, dtype=torch.float64, device=cuda_device))
    liked = [sorted(rng.choice(n, int(m), replace=False).tolist()) for m in rng.integers(1, 9, 200)]
    rated = [sorted(set(l) | set(rng.choice(n, 5).tolist())) for l in liked]
    st = HostStager(cuda_device)
    lo = csr_from_lists(liked, cuda_device, st)
    eo = csr_from_lists(rated, cuda_device, st)
    assert lo.checked_for(0, n)
    s, r = ebt.score_topk(cat, k, liked=lo, exclude=eo)
    s2, r2 = ebt.score_topk(cat, k, liked=liked, exclude=rated)
    assert torch.equal(r, r2) and torch.equal(s, s2)
    # a plain tuple is not known checked: the C entry reads it back (the host-scale path) --
    # the device 1/L scale gives the same bits
    s3, r3 = ebt.score_topk(cat, k, liked=(lo[0], lo[1]), exclude=eo)
    assert torch.equal(r, r3) and torch.equal(s, s3)
    s_ref, r_ref = R.liked_topk(x, liked, k, exclude=rated)
    assert np.array_equal(r.cpu().numpy(), r_ref)
    np.testing.assert_allclose(s.cpu().numpy(), s_ref, rtol=0, atol=1e-12)
