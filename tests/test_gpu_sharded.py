"""GPU: the two-phase sharded top-k (distributed.score_topk_sharded) on ONE GPU, R ranks
simulated by R threads whose collectives are an in-process exchange (same tensors, same
order as all_gather_into_tensor / all_reduce). Every rank's answer must equal the single-catalog
score_topk and the float64 oracle; the torch.distributed calls themselves are covered by
test_dist_gloo.py."""
import threading

import numpy as np
import pytest
import torch

from inputs import gaussian
from oracle import restatement as R

pytestmark = pytest.mark.gpu


class ThreadCollectives:
    def __init__(self, rank, shared):
        self.rank, self.s = rank, shared
        self.world = shared["world"]

    def _exchange(self, t):
        self.s["slots"][self.rank] = t.clone()
        self.s["barrier"].wait()
        vals = list(self.s["slots"])
        self.s["barrier"].wait()
        return vals

    def all_gather(self, t):
        return torch.stack(self._exchange(t))

    def all_reduce_sum(self, t):
        t.copy_(torch.stack(self._exchange(t)).sum(0))
        return t

    def all_reduce_max(self, t):
        t.copy_(torch.stack(self._exchange(t)).max(0).values)
        return t


def _run_sharded(full, world, fn, cuts=None):
    """fn(rank, catalog_shard, collectives) in `world` threads; returns the per-rank results.
    cuts: explicit shard boundaries [0, ..., n] (default: shard_range)."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import shard_range
    n = full.shape[0]
    shared = {"world": world, "slots": [None] * world, "barrier": threading.Barrier(world)}
    cats = []
    for r in range(world):
        a, b = (cuts[r], cuts[r + 1]) if cuts is not None else shard_range(n, r, world)
        cats.append(ebt.Catalog(full[a:b].contiguous(), row_offset=a, n_global=n))
    out, errs = [None] * world, []

    def body(r):
        try:
            out[r] = fn(r, cats[r], ThreadCollectives(r, shared))
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            shared["barrier"].abort()
    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("world,dt", [(3, "f32"), (2, "bf16")])
def test_two_phase_matches_single_and_oracle(cuda_device, world, dt):
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import score_topk_sharded
    from test_gpu_parity import TORCH_DT, _t, assert_topk_equal
    n, d, B, k = 150_000, 256, 70, 50
    c = gaussian(31, n, d, dt)
    q = gaussian(32, B, d, dt)
    rng = np.random.default_rng(33)
    excl = [sorted(rng.choice(n, 300, replace=False).tolist()) for _ in range(B)]
    full = _t(c, dt, cuda_device)
    qt = _t(q, dt, cuda_device)
    res = _run_sharded(full, world, lambda r, cat, coll: score_topk_sharded(
        cat, k, queries=qt, exclude=excl, collectives=coll))
    single = ebt.score_topk(ebt.Catalog(full), k, queries=qt, exclude=excl)
    for s, r in res:
        assert torch.equal(r, single[1])
        torch.testing.assert_close(s, single[0], rtol=0, atol=0)
    sample = [0, 35, 69]
    s_ref, r_ref = R.cosine_topk(q[sample].astype(np.float64), c.astype(np.float64), k,
                                 [excl[i] for i in sample])
    assert_topk_equal(res[0][0][sample], res[0][1][sample], s_ref, r_ref)


def test_two_phase_liked_queries(cuda_device):
    """Liked rows spread over shards: the all-reduce of partial sums completes the mean."""
    from robot_ebert_amd.distributed import score_topk_sharded
    from test_gpu_parity import _t, assert_topk_equal
    n, d, k = 20_000, 64, 30
    c = gaussian(41, n, d, "f64")
    liked = [[1, 2, 19_999], [10_000], [5, 6_000, 12_000, 18_000]]
    rated = [l + [7, 8] for l in liked]
    full = _t(c, "f64", cuda_device)
    res = _run_sharded(full, 3, lambda r, cat, coll: score_topk_sharded(
        cat, k, liked=liked, exclude=rated, collectives=coll))
    want_s, want_r = R.liked_topk(c, liked, k, rated)
    for s, r in res:
        assert_topk_equal(s, r, want_s, want_r)


def test_two_phase_overflow_and_retry(cuda_device):
    """Scores rising with the row id overflow the fused screen's hit slots on the last shard:
    the flag is all-reduced, every rank reruns that query unfused, the answer stays exact."""
    from robot_ebert_amd.distributed import score_topk_sharded
    from test_gpu_parity import _t, assert_topk_equal
    n, d, k = 300_000, 64, 16
    rng = np.random.default_rng(9)
    q = rng.standard_normal((2, d))
    t = (np.arange(n) / n)[:, None]
    c = q[0][None, :] * t + rng.standard_normal((n, d)) * (1.0 - t) * 0.5
    full = _t(c, "f64", cuda_device)
    qt = _t(q, "f64", cuda_device)
    res = _run_sharded(full, 2, lambda r, cat, coll: score_topk_sharded(
        cat, k, queries=qt, collectives=coll))
    s_ref, r_ref = R.cosine_topk(q, c, k)
    for s, r in res:
        assert_topk_equal(s, r, s_ref, r_ref)


def cat_has(row, r, n, world):
    from robot_ebert_amd.distributed import shard_range
    a, b = shard_range(n, r, world)
    return a <= row < b


@pytest.mark.parametrize("world,dt", [(4, "f32"), (2, "bf16")])
def test_per_shard_global_cut_matches_single(cuda_device, world, dt):
    """score_topk_sharded_local: each shard rescores only rows above the all-reduced floor
    (t_floor), leaving NaN / -1 slots; the merged answer equals the single-GPU one exactly."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import score_topk_sharded_local
    from robot_ebert_amd.search import union_floor
    from test_gpu_parity import _t, assert_topk_equal
    n, d, B, k = 160_000, 256, 64, 100
    c = gaussian(51, n, d, dt)
    q = gaussian(52, B, d, dt)
    rng = np.random.default_rng(53)
    excl = [sorted(rng.choice(n, 200, replace=False).tolist()) for _ in range(B)]
    full = _t(c, dt, cuda_device)
    qt = _t(q, dt, cuda_device)
    partial = {}

    def body(r, cat, coll):
        out = score_topk_sharded_local(cat, k, queries=qt, exclude=excl, collectives=coll)
        # the shard's own (cut) list, for the empty-slot checks below
        partial[r] = ebt.score_topk(cat, k, queries=qt, exclude=excl,
                                    t_floor_hook=lambda v, e: union_floor(
                                        coll.all_gather(v), coll.all_gather(e), k))
        return out
    res = _run_sharded(full, world, body)
    single = ebt.score_topk(ebt.Catalog(full), k, queries=qt, exclude=excl)
    for s, r in res:
        assert torch.equal(r, single[1])
        torch.testing.assert_close(s, single[0], rtol=0, atol=0)
    # the cut removed work: a shard keeps about k/world + (rows in the eps band) of its top k
    empty = sum(int((partial[r][1] < 0).sum()) for r in range(world))
    assert empty >= B * k * (world - 1) // 4
    glob = set(map(tuple, [(b, int(x)) for b in range(B) for x in single[1][b].tolist()]))
    for r in range(world):
        ps, pr = partial[r]
        valid = pr >= 0
        assert bool(torch.isnan(ps[~valid]).all())
        # the kept rows are a prefix, and every kept row within the global k-th score's
        # neighbourhood: a row of the global top k is never cut
        assert bool((valid[:, 1:] <= valid[:, :-1]).all())
        kept = set((b, int(x)) for b in range(B) for x in pr[b][valid[b]].tolist())
        mine = set(p for p in glob if cat_has(p[1], r, n, world))
        assert mine <= kept
    sample = [0, 63]
    s_ref, r_ref = R.cosine_topk(q[sample].astype(np.float64), c.astype(np.float64), k,
                                 [excl[i] for i in sample])
    assert_topk_equal(res[0][0][sample], res[0][1][sample], s_ref, r_ref)


def test_per_shard_global_cut_uneven_shards(cuda_device):
    """A shard smaller than k contributes no floor (its list ends in -inf / holds < k rows);
    liked queries spread over the shards; the merge still equals the oracle."""
    from robot_ebert_amd.distributed import score_topk_sharded_local
    from test_gpu_parity import _t, assert_topk_equal
    n, d, k = 30_000, 64, 40
    c = gaussian(61, n, d, "f64")
    liked = [[1, 2, 29_999], [29_990], [5, 6_000, 12_000, 29_995]]
    rated = [l + [7, 8, 29_980] for l in liked]
    full = _t(c, "f64", cuda_device)
    cuts = [0, 14_000, 29_975, n]   # the last shard holds 25 < k rows
    res = _run_sharded(full, 3, lambda r, cat, coll: score_topk_sharded_local(
        cat, k, liked=liked, exclude=rated, collectives=coll), cuts=cuts)
    want_s, want_r = R.liked_topk(c, liked, k, rated)
    for s, r in res:
        assert_topk_equal(s, r, want_s, want_r)


def test_per_shard_global_cut_overflow_retry(cuda_device):
    """Overflowed fused lists under the global cut rerun unfused locally (no collective)."""
    from robot_ebert_amd.distributed import score_topk_sharded_local
    from test_gpu_parity import _t, assert_topk_equal
    n, d, k = 300_000, 64, 16
    rng = np.random.default_rng(9)
    q = rng.standard_normal((2, d))
    t = (np.arange(n) / n)[:, None]
    c = q[0][None, :] * t + rng.standard_normal((n, d)) * (1.0 - t) * 0.5
    full = _t(c, "f64", cuda_device)
    qt = _t(q, "f64", cuda_device)
    res = _run_sharded(full, 2, lambda r, cat, coll: score_topk_sharded_local(
        cat, k, queries=qt, collectives=coll))
    s_ref, r_ref = R.cosine_topk(q, c, k)
    for s, r in res:
        assert_topk_equal(s, r, s_ref, r_ref)


def _spy(monkeypatch, module, name, log):
    orig = getattr(module, name)

    def wrapper(*a, **kw):
        log.append(kw.get("flags", a[8] if name == "run_pipeline" and len(a) > 8 else None))
        return orig(*a, **kw)
    monkeypatch.setattr(module, name, wrapper)


@pytest.mark.parametrize("world,dt", [(2, "f32"), (4, "bf16")])
def test_shared_threshold_matches_single(cuda_device, monkeypatch, world, dt):
    """score_topk_sharded_local screens every shard at ONE catalog-wide threshold (the
    all-gathered sample maxima of all shards, ebt_cosine_sample + ebt_pool_kth +
    ebt_cosine_screen_at): the merged answer equals the single-GPU one and the oracle."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd import search
    from robot_ebert_amd.distributed import score_topk_sharded_local, shared_sample_tiles
    from test_gpu_parity import _t, assert_topk_equal
    n, d, B, k = 400_000, 128, 300, 50
    assert shared_sample_tiles(n, world, search.pad_batch(B)) > 0
    c = gaussian(71, n, d, dt)
    q = gaussian(72, B, d, dt)
    rng = np.random.default_rng(73)
    excl = [sorted(rng.choice(n, 100, replace=False).tolist()) for _ in range(B)]
    full = _t(c, dt, cuda_device)
    qt = _t(q, dt, cuda_device)
    calls = []
    _spy(monkeypatch, search, "screen_at", calls)
    res = _run_sharded(full, world, lambda r, cat, coll: score_topk_sharded_local(
        cat, k, queries=qt, exclude=excl, collectives=coll))
    assert len(calls) == world          # every shard screened at the shared threshold
    single = ebt.score_topk(ebt.Catalog(full), k, queries=qt, exclude=excl)
    for s, r in res:
        assert torch.equal(r, single[1])
        torch.testing.assert_close(s, single[0], rtol=0, atol=0)
    sample = [0, 150, 299]
    s_ref, r_ref = R.cosine_topk(q[sample].astype(np.float64), c.astype(np.float64), k,
                                 [excl[i] for i in sample])
    assert_topk_equal(res[0][0][sample], res[0][1][sample], s_ref, r_ref)


def test_shared_threshold_too_high_reruns(cuda_device, monkeypatch):
    """An adversarial catalog whose only high rows sit exactly in the sampled subgroups (20 of
    them, k = 50): the shared threshold lands above the k-th score, every query fails the
    theta <= t_floor - eps check and is rerun unfused on its shard; the answer stays exact."""
    from robot_ebert_amd import search
    from robot_ebert_amd.distributed import score_topk_sharded_local, shared_sample_tiles
    from test_gpu_parity import _t, assert_topk_equal
    n, d, B, k, world = 200_000, 64, 256, 50, 2
    tiles = shared_sample_tiles(n, world, search.pad_batch(B))
    assert tiles > 0
    rng = np.random.default_rng(81)
    q0 = rng.standard_normal(d)
    c = rng.standard_normal((n, d))
    stride = (n // world // 256) // tiles
    stride -= 1 if stride > 1 and stride % 2 == 0 else 0   # search.sample_maxima's odd stride
    boosted = [t * stride * 256 + 64 * s for t in range(5) for s in range(4)]   # shard 0
    c[boosted] = q0[None, :] + 0.3 * rng.standard_normal((len(boosted), d))
    q = q0[None, :] + 0.05 * rng.standard_normal((B, d))
    full = _t(c, "f64", cuda_device)
    qt = _t(q, "f64", cuda_device)
    reruns = []
    _spy(monkeypatch, search, "run_pipeline", reruns)
    res = _run_sharded(full, world, lambda r, cat, coll: score_topk_sharded_local(
        cat, k, queries=qt, collectives=coll))
    assert reruns, "the too-high threshold was not caught"
    sample = [0, 77, 255]
    s_ref, r_ref = R.cosine_topk(q[sample], c, k)
    for s, r in res:
        assert_topk_equal(s[sample], r[sample], s_ref, r_ref)
    s_all, r_all = R.cosine_topk(q, c, k)
    assert np.array_equal(res[0][1].cpu().numpy(), r_all)


@pytest.mark.parametrize("world", [2, 8])
def test_staged_two_in_flight_matches_single(cuda_device, world):
    """run_sharded_steps (bench.py's N > 1 loop): batches interleaved stage by stage, two in
    flight, every collective started in stage order on every rank; each batch's merged answer
    equals the single-GPU one. Different queries per batch catch any mix-up between batches."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import run_sharded_steps, score_topk_sharded_local_stages
    from test_gpu_parity import _t
    n, d, B, k, steps = 240_000, 128, 300, 50, 4
    c = gaussian(91, n, d, "f32")
    qs = [gaussian(92 + i, B, d, "f32") for i in range(steps)]
    full = _t(c, "f32", cuda_device)
    qts = [_t(q, "f32", cuda_device) for q in qs]

    def body(r, cat, coll):
        it = iter(range(steps))
        seen = []

        def make():
            i = next(it)
            seen.append(i)
            return score_topk_sharded_local_stages(cat, k, queries=qts[i], collectives=coll)
        outs = []
        # capture every batch's result: drive run_sharded_steps over 1..steps batches
        for m in range(1, steps + 1):
            it = iter(range(m))
            outs.append(run_sharded_steps(make, m))
        return outs
    res = _run_sharded(full, world, body)
    cat = ebt.Catalog(full)
    for m in range(1, steps + 1):
        s_ref, r_ref = ebt.score_topk(cat, k, queries=qts[m - 1])
        for r in range(world):
            s, rr = res[r][m - 1]
            assert torch.equal(rr, r_ref)
            torch.testing.assert_close(s, s_ref, rtol=0, atol=0)


def test_rccl_world1_staged_path(cuda_device):
    """The real torch.distributed calls of bench.py's N > 1 loop over RCCL ("nccl"), on a
    one-rank group (the only group one GPU allows): async all-gathers with deferred waits
    (TorchCollectives.all_gather_start), the floor hook, an explicit shared-threshold hook and
    the staged two-in-flight driver; the answers equal the single-GPU path."""
    import socket
    import torch.distributed as dist
    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import (TorchCollectives, _shared_theta, run_sharded_steps,
                                             score_topk_sharded_local_stages, shared_sample_tiles)
    from test_gpu_parity import _t
    n, d, B, k = 150_000, 128, 300, 50
    c = gaussian(101, n, d, "f32")
    qs = [_t(gaussian(102 + i, B, d, "f32"), "f32", cuda_device) for i in range(3)]
    cat = ebt.Catalog(_t(c, "f32", cuda_device))
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=cuda_device)
    try:
        coll = TorchCollectives()
        tiles = shared_sample_tiles(n * 2, 2, 512)   # a sample size the 2-rank layout would use
        assert tiles > 0
        it = iter(range(3))

        def make():
            i = next(it)
            return score_topk_sharded_local_stages(
                cat, k, queries=qs[i], collectives=coll,
                theta_hook=lambda qb, kp: _shared_theta(coll, cat, qb, kp, tiles))
        s, r = run_sharded_steps(make, 3)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    s_ref, r_ref = ebt.score_topk(cat, k, queries=qs[2])
    assert torch.equal(r, r_ref)
    torch.testing.assert_close(s, s_ref, rtol=0, atol=0)


def test_shared_threshold_liked_users(cuda_device):
    """The collaborative path (liked rows spread over the shards, all-reduced partial sums)
    through the staged driver with the shared threshold and exclusions of the rated rows."""
    from robot_ebert_amd.distributed import (run_sharded_steps, score_topk_sharded_local_stages,
                                             shared_sample_tiles)
    from robot_ebert_amd.search import pad_batch
    from test_gpu_parity import _t, assert_topk_equal
    n, d, k, world, B = 200_000, 64, 20, 2, 150
    assert shared_sample_tiles(n, world, pad_batch(B)) > 0
    c = gaussian(111, n, d, "f64")
    rng = np.random.default_rng(112)
    liked = [sorted(rng.choice(n, int(rng.integers(1, 12)), replace=False).tolist())
             for _ in range(B)]
    rated = [sorted(set(l) | set(rng.choice(n, 30, replace=False).tolist())) for l in liked]
    full = _t(c, "f64", cuda_device)
    res = _run_sharded(full, world, lambda r, cat, coll: run_sharded_steps(
        lambda: score_topk_sharded_local_stages(cat, k, liked=liked, exclude=rated,
                                                collectives=coll), 2))
    sample = [0, 75, 149]
    want_s, want_r = R.liked_topk(c, [liked[i] for i in sample], k, [rated[i] for i in sample])
    for s, r in res:
        assert_topk_equal(s[sample], r[sample], want_s, want_r)


@pytest.mark.parametrize("R,k,kk", [(8, 100, 100), (3, 7, 16), (2, 1000, 1000), (64, 10, 32),
                                    (33, 20, 64), (8, 1000, 1000), (9, 1000, 1000)])
def test_union_floor_kernel_matches_torch(cuda_device, R, k, kk):
    """ebt_union_floor (bisection over 64-bit keys: keys in registers, one wave per query up to
    2048 values, one workgroup up to 8192, the strided form beyond) equals the torch
    restatement (the k-th largest of approx - eps over all shards), with -inf padding, NaNs and
    ties."""
    from robot_ebert_amd.search import union_floor_gathered
    from floor_ref import union_floor_torch as union_floor
    B = 333
    g = torch.Generator().manual_seed(R * 1000 + k)
    vals = torch.randn((R, B, kk), generator=g) * 0.03
    vals[:, :, kk // 2:] = float("-inf")                 # short lists
    vals[0, :5, 0] = float("nan")
    vals[:, 7, :] = 0.25                                 # ties
    eps = torch.rand((R, B), generator=g) * 1e-3
    want = union_floor(vals, eps, k)                     # CPU tensors: the torch form
    got = union_floor_gathered(torch.cat([vals, eps[:, :, None]], 2).to(cuda_device), k)
    assert torch.equal(got.cpu(), want)


def test_rccl_comm_capi_world1(cuda_device):
    """bench.py's N > 1 C-ABI path on the one group one GPU allows: libebert's own RCCL
    communicator (ebt_rccl_unique_id broadcast through a torch "nccl" group, ebt_rccl_comm_init,
    ncclAllGather inside ebt_cosine_topk_sharded_*) driving ShardedTopk with three batches in
    flight; the answers equal the single-GPU path, and a direct ebt_rccl_all_gather round-trips
    a buffer."""
    import socket
    import torch.distributed as dist
    import robot_ebert_amd as ebt
    from robot_ebert_amd import _lib
    from robot_ebert_amd.distributed import RcclComm, ShardedTopk
    from test_gpu_parity import _t
    n, d, B, k = 150_000, 128, 300, 50
    cat = ebt.Catalog(_t(gaussian(111, n, d, "f32"), "f32", cuda_device))
    q = _t(gaussian(112, B, d, "f32"), "f32", cuda_device)
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=cuda_device)
    try:
        rc = RcclComm()
        try:
            x = torch.arange(1000, dtype=torch.int32, device=cuda_device)
            y = torch.zeros_like(x)
            _lib.call("ebt_rccl_all_gather", rc.handle, _lib.ptr(x), _lib.ptr(y), 4000,
                      _lib.stream_of(cuda_device))
            torch.cuda.synchronize()
            assert torch.equal(x, y)
            z = torch.linspace(-1, 1, 777, dtype=torch.float64, device=cuda_device)
            z0 = z.clone()
            _lib.call("ebt_rccl_all_reduce_f64", rc.handle, _lib.ptr(z), 777,
                      _lib.stream_of(cuda_device))
            torch.cuda.synchronize()
            assert torch.equal(z, z0)   # one rank: the sum is its own buffer
            eng = ShardedTopk(cat, k, B, rc)
            s, r = eng.run(4, q)
            torch.cuda.synchronize()
        finally:
            rc.close()
    finally:
        dist.destroy_process_group()
    s_ref, r_ref = ebt.score_topk(cat, k, queries=q)
    assert torch.equal(r, r_ref)
    assert torch.equal(s, s_ref)
