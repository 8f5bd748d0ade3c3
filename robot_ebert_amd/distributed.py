"""Row-sharded catalog over the GPUs of one node (one process per GPU, torch.distributed).

The reference scales only by Cloud Run replicas (README.md:78-82) and has no collective. Here
the catalog rows are split into contiguous blocks, rank r holding rows
[shard_range(n, r, R)), and every rank screens the full query batch against its shard (global row
ids via ``row_offset``). Two exchange patterns:

* ``score_topk_sharded`` (two-phase): every rank screens its shard
  (``ebt_cosine_screen``: approx k' candidates, no rescore), ONE all-gather of the candidate lists
  (B x k' f32 + i64 over RCCL/xGMI), every rank keeps the k' best of all shards, computes the
  exact float64 scores of the merged candidates IT owns (``ebt_rescore_owned``), ONE all-reduce
  (SUM, B x k' f64) completes them, and ``ebt_finalize_topk`` sorts and certifies. Each candidate
  row is gathered and rescored once in the whole job instead of once per shard. Simulated on one
  GPU (tools/shard_sim.py) its per-rank compute at 8 ranks of C3 is within 2 % of the other
  path's while it moves more data (B x k' candidates + a B x k' all-reduce), so it is offered,
  not the bench default.
* ``score_topk_sharded_local`` (bench.py's N > 1 step): every rank runs the full single-GPU path
  on its shard and the per-shard exact top-k are all-gathered and merged (``ebt_merge_topk``):
  one collective of B x k (f64, i64) per step.

For the collaborative path the liked rows of a user live on several shards: each rank sums its
local normalised liked rows and one all-reduce (SUM) of the B x d float64 partial sums completes
the query vectors before screening. Retries (uncertified / overflowed queries) are decided from
all-gathered data, so every rank takes the same retry and the collectives stay in lockstep.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _lib
from ._lib import EbertError, call, ptr, region, stream_of
from .catalog import Catalog
from .search import (KPRIME_MAX, MERGE_WAVE_KMAX, _round_up, csr_from_lists, csr_subset,
                     default_kprime, merge_topk, pad_batch, pool_kth, prepare_queries, run_screen,
                     sample_maxima, score_topk, score_topk_finish, score_topk_stages,
                     score_topk_submit, spec_rank, union_floor_gathered)

SAMPLE_TILES_MAX = 64   # per shard, as the single-GPU speculative screen (api.hip spec_params)
# Larger shards screen at their own sample threshold: there the shard's first segment raises
# its threshold (list k-th - 2 eps) soon enough, and the shared threshold's uniform hits cost
# as much as they save (round 5, tools/rank_sim_capi.py replays of C3, two runs each: 4 ranks
# 2.689 vs 2.734 ms per step with the shared threshold, 2 ranks 5.251 vs 5.214 ms; round 3's
# shard_sim: 8 ranks -3 %). driver.hip EBT_SH_SHARED_MAX is the same limit.
SHARED_MAX_SHARD_ROWS = 300_000


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block of rows owned by `rank` (sizes differ by at most one row)."""
    base, rem = divmod(n, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def gather_partials(scores: torch.Tensor, rows: torch.Tensor,
                    group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather the [B, k] partial results of every rank -> [R, B, k] (rank order)."""
    world = dist.get_world_size(group)
    B = scores.shape[0]
    # concatenated along dim 0 (the layout every backend accepts), viewed as [R, B, k]
    gs = torch.empty((world * B,) + tuple(scores.shape[1:]), dtype=scores.dtype,
                     device=scores.device)
    gr = torch.empty((world * B,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    dist.all_gather_into_tensor(gs, scores.contiguous(), group=group)
    dist.all_gather_into_tensor(gr, rows.contiguous(), group=group)
    return gs.view((world,) + tuple(scores.shape)), gr.view((world,) + tuple(rows.shape))


def split_liked(liked: Sequence[Sequence[int]], begin: int, end: int):
    """Per-user liked rows that fall into [begin, end), plus every user's total count."""
    local = [[r for r in l if begin <= r < end] for l in liked]
    counts = [len(l) for l in liked]
    return local, counts


class TorchCollectives:
    """The three collectives the two-phase path uses, over a torch.distributed group (RCCL on
    MI355X: backend "nccl"; gloo on CPU)."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None) -> None:
        self.group = group
        self.world = dist.get_world_size(group)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out.view((self.world,) + tuple(t.shape))

    def all_gather_start(self, t: torch.Tensor):
        """Start an all-gather without making the stream wait for it; the returned callable
        makes the CURRENT stream wait (work.wait()) and returns the [R, ...] result. Kernels
        enqueued in between run while the collective is in flight."""
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        src = t.contiguous()
        work = dist.all_gather_into_tensor(out, src, group=self.group, async_op=True)
        shape = (self.world,) + tuple(t.shape)

        def wait():
            work.wait()
            _ = src  # keep the source alive until the collective has finished
            return out.view(shape)
        return wait

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t


def _liked_queries(catalog: Catalog, liked, coll):
    local, counts = split_liked(liked, catalog.row_offset, catalog.row_offset + catalog.n)
    dev = catalog.device
    return (csr_from_lists(local, dev), torch.tensor(counts, dtype=torch.int64, device=dev),
            lambda q64: coll.all_reduce_sum(q64))


def _two_phase(catalog: Catalog, qb, k: int, kprime: int, exclude, chunk_rows, timer, flags,
               coll):
    dev = catalog.device
    st = stream_of(dev)
    B = qb.B
    lv, lr, ovf, eps = run_screen(catalog, qb, k, kprime, exclude, chunk_rows, timer, flags)
    R = coll.world
    gv = coll.all_gather(lv)        # [R, B, k']
    gr = coll.all_gather(lr)
    ovf = coll.all_reduce_max(ovf)
    # every rank: the k' best of all shards (rows are the select's indices)
    vals = gv.permute(1, 0, 2).reshape(B, R * kprime).contiguous()
    rows = gr.permute(1, 0, 2).reshape(B, R * kprime).contiguous()
    mv = torch.empty((B, kprime), dtype=torch.float32, device=dev)
    mr = torch.empty((B, kprime), dtype=torch.int64, device=dev)
    call("ebt_select_topk", ptr(vals), ptr(rows), R * kprime, B, R * kprime, 0, kprime, 1,
         ptr(mv), ptr(mr), kprime, st)
    exact = torch.empty((B, kprime), dtype=torch.float64, device=dev)
    call("ebt_rescore_owned", ptr(qb.q64), B, catalog.d, ptr(catalog.data), catalog.dtype_code,
         catalog.ld, ptr(catalog.gnorm), catalog.row_offset, catalog.n, ptr(mv), ptr(mr), kprime,
         k, ptr(eps), ptr(exact), st)
    exact = coll.all_reduce_sum(exact)
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    cert = torch.empty(B, dtype=torch.int32, device=dev)
    call("ebt_finalize_topk", ptr(mv), ptr(mr), ptr(exact), B, kprime, k, catalog.n_global,
         ptr(eps), ptr(ovf), ptr(out_s), ptr(out_r), ptr(cert), st)
    return out_s, out_r, cert


def score_topk_sharded(catalog: Catalog, k: int, queries: Optional[torch.Tensor] = None,
                       liked: Optional[Sequence[Sequence[int]]] = None,
                       exclude=None, group: Optional[dist.ProcessGroup] = None,
                       kprime: Optional[int] = None, chunk_rows: Optional[int] = None,
                       timer=None, fuse: bool = True, collectives=None
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Global top-k over a row-sharded catalog, two-phase (see the module doc); every rank
    returns the same (scores f64 [B, k], GLOBAL rows i64 [B, k]). ``exclude``: per-query GLOBAL
    rows (lists or device CSR). ``collectives`` replaces the torch.distributed calls (tests)."""
    coll = collectives if collectives is not None else TorchCollectives(group)
    dev = catalog.device
    if k < 1:
        raise EbertError("k must be >= 1")
    if exclude is not None and not isinstance(exclude, tuple):
        exclude = csr_from_lists(exclude, dev)
    if liked is not None:
        liked_csr, counts, hook = _liked_queries(catalog, liked, coll)
        qb = prepare_queries(catalog, liked=liked_csr, liked_counts=counts, liked_sum_hook=hook)
    else:
        qb = prepare_queries(catalog, queries=queries)
    n_cap = _round_up(catalog.n_global, 4)
    k_eff = min(k, catalog.n_global)
    if k_eff > KPRIME_MAX:
        raise EbertError(f"k={k} > {KPRIME_MAX} is not supported")
    kp = kprime or default_kprime(catalog, k_eff)
    kp = max(_round_up(k_eff, 4), min(_round_up(kp, 4), n_cap, KPRIME_MAX))
    flags = 0 if fuse else _lib.EBT_FLAG_NO_FUSE
    s, r, cert = _two_phase(catalog, qb, k_eff, kp, exclude, chunk_rows, timer, flags, coll)
    while True:  # identical certificates on every rank -> identical retries
        flat = cert.cpu()
        over = torch.nonzero(flat == -1).flatten().to(dev)
        bad = torch.nonzero(flat == 0).flatten().to(dev)
        if over.numel() == 0 and bad.numel() == 0:
            break
        if over.numel():
            sub_ex = csr_subset(exclude[0], exclude[1], over) if exclude is not None else None
            s2, r2, c2 = _two_phase(catalog, qb.subset(over), k_eff, kp, sub_ex, chunk_rows,
                                    timer, _lib.EBT_FLAG_NO_FUSE, coll)
            s[over], r[over], cert[over] = s2, r2, c2
            continue
        widen = kp < min(n_cap, KPRIME_MAX)
        if not widen and flags & _lib.EBT_FLAG_EXACT:
            raise EbertError(f"{bad.numel()} queries could not be certified at k'={kp} "
                             "(more than k' rows tie with the k-th score at f32 precision)")
        if widen:
            kp = min(kp * 4, n_cap, KPRIME_MAX)
        else:
            flags = _lib.EBT_FLAG_EXACT
            kp = max(_round_up(k_eff, 4), min(_round_up(default_kprime(catalog, k_eff), 4),
                                              n_cap, KPRIME_MAX))
        sub_ex = csr_subset(exclude[0], exclude[1], bad) if exclude is not None else None
        s2, r2, c2 = _two_phase(catalog, qb.subset(bad), k_eff, kp, sub_ex, chunk_rows, timer,
                                flags, coll)
        s[bad], r[bad], cert[bad] = s2, r2, c2
    if k_eff < k:
        pad_s = torch.full((qb.B, k - k_eff), float("nan"), dtype=torch.float64, device=dev)
        pad_r = torch.full((qb.B, k - k_eff), -1, dtype=torch.int64, device=dev)
        s, r = torch.cat([s, pad_s], 1), torch.cat([r, pad_r], 1)
    return s, r


def _gather_start(coll, t: torch.Tensor):
    """coll.all_gather_start when the collectives offer it, else a completed all-gather."""
    if hasattr(coll, "all_gather_start"):
        return coll.all_gather_start(t)
    g = coll.all_gather(t)
    return lambda: g


def shard_list_width(k: int, world: int) -> int:
    """min(k, ceil(1.5 k / world) + 8): the entries per query a shard sends for the floor (its
    widest expected share of the global top k, with margin), and the packed results' capacity
    per query (include/ebert.h ebt_shard_list_width)."""
    return int(_lib.load().ebt_shard_list_width(k, world))


def floor_send(vals: torch.Tensor, eps: Optional[torch.Tensor], w: int) -> torch.Tensor:
    """[B, w + 1] f32: the w largest of each row of vals (a partitioned list is fine), -inf
    padded, then eps (-inf when None) (ebt_floor_pack)."""
    B, ld = vals.shape
    vals = vals.contiguous()
    out = torch.empty((B, w + 1), dtype=torch.float32, device=vals.device)
    call("ebt_floor_pack", ptr(vals), ld, B, ld, w,
         ptr(eps.contiguous()) if eps is not None else None, ptr(out), stream_of(vals.device))
    return out


def _gathered_floor(coll, vals: torch.Tensor, eps: torch.Tensor, k: int, timer=None):
    """union_floor over every shard's (w best approx, eps), w = shard_list_width(k, R), in ONE
    all-gather ([B, w+1] f32; the k-th largest over a subset of the values is still a lower
    bound); returns a future (the gather runs while the caller enqueues other work)."""
    with region(timer, "small", vals.device):
        send = floor_send(vals, eps, shard_list_width(k, coll.world))
    wait = _gather_start(coll, send)
    dev = vals.device

    def floor():
        with region(timer, "collective_wait", dev):
            g = wait()
        with region(timer, "small", dev):
            return union_floor_gathered(g, k)
    return floor


def shared_sample_tiles(n_global: int, world: int, B_pad: int) -> int:
    """256-row sample tiles per shard for the shared screening threshold, 0 = not used. Depends
    only on (n_global, world, B_pad), so every rank takes the same decision (the threshold's
    all-gather is a collective). The single-GPU rule (api.hip spec_params: <= 64 tiles, <= 1/24
    of the rows, whole rounds of 256 workgroups when that keeps >= 8) on the largest shard."""
    if world < 2 or B_pad % 256 != 0 or -(-n_global // world) > SHARED_MAX_SHARD_ROWS:
        return 0
    full = -(-n_global // world) // 256
    # about the single-GPU sample in total (64 tiles over all shards, >= 4 per shard): a larger
    # pooled sample tightens theta little but costs every shard its GEMM and a wider pool_kth
    P = min(SAMPLE_TILES_MAX, full // 24, max(4, -(-SAMPLE_TILES_MAX // world)))
    per = max(1, 256 // (B_pad // 256))
    if P // per * per >= 8:
        P = P // per * per
    # less than one round of the persistent grid takes a round's time anyway: fill it
    # (only within the sample's caps: ebt_pool_kth takes at most 2048 maxima per query)
    if P < per and per <= full // 6 and per <= SAMPLE_TILES_MAX and world * 4 * per <= 2048:
        P = per
    return P if P >= 1 and world * P >= 8 else 0


def sample_send_width(kp_glob: int, tiles: int, world: int, n_global: int) -> int:
    """J: how many of its 4 * tiles sample maxima per query a shard sends. theta is the j-th
    largest of all shards' maxima with j <= J (J from the catalog-wide k', the same on every
    rank), and the j-th largest of the union of each shard's J largest is that same value.
    0 = no shared threshold (the sample would decide nothing). driver.hip shard_layout."""
    m_total = 256 * tiles * world
    J = spec_rank(kp_glob * m_total / max(n_global, 1))
    if J > world * 4 * tiles // 2:
        return 0
    return min(J, 4 * tiles)


def _shared_theta(coll, catalog: Catalog, qb, kprime: int, tiles: int, timer=None,
                  kp_glob: Optional[int] = None):
    """Catalog-wide screening threshold: every shard's sample maxima (ebt_cosine_sample), its J
    largest per query (sample_send_width: ebt_floor_pack), ONE all-gather ([R, B, J + 1] f32),
    theta = the j-th largest of all of them (ebt_pool_kth), j from the Poisson bound of
    spec_params with the k'-th best of the WHOLE catalog as the target. Each shard then keeps
    ~(its share of) k' j / lambda rows per query instead of ~k' j / lambda of its own, and one
    filter launch covers it. Returns a future of (theta [B_pad], expected hits per query on this
    shard) or None (every rank alike)."""
    J = sample_send_width(kp_glob or kprime, tiles, coll.world, catalog.n_global)
    pooled = local_sample(catalog, qb, tiles, timer)                       # [B, 4 tiles]
    with region(timer, "small", catalog.device):
        send = floor_send(pooled, None, J) if J else pooled
    wait = _gather_start(coll, send)                                       # [R, B, J + 1]

    def theta():
        with region(timer, "collective_wait", catalog.device):
            g = wait()
        with region(timer, "small", catalog.device):
            return theta_from_samples(g, qb, kprime, tiles, catalog.n_global, catalog.n,
                                      sent=J or 4 * tiles)
    return theta


def local_sample(catalog: Catalog, qb, tiles: int, timer=None) -> torch.Tensor:
    """This shard's part of the shared threshold: [B, 4 tiles] f32 sample maxima (-inf where a
    shard too small for `tiles` full tiles has none)."""
    B, G = qb.B, 4 * tiles
    pooled = torch.full((B, G), float("-inf"), dtype=torch.float32, device=catalog.device)
    own = min(tiles, catalog.n // 256)
    if own >= 1:
        pooled[:, :4 * own] = sample_maxima(catalog, qb, own, timer)[:B]
    return pooled


def theta_from_samples(g: torch.Tensor, qb, kprime: int, tiles: int, n_global: int,
                       n_local: int, sent: Optional[int] = None):
    """(theta [B_pad], expected hits per query on an n_local-row shard) from the gathered
    [R, B, G] maxima, or None when the sample is too small to say anything. `sent` = how many
    maxima per query each shard sent (J of sample_send_width; the gathered rows of a packed
    send carry one extra -inf column, G = J + 1): the j-th largest of the union is exact for
    j <= sent, and for any j <= RG / 2 when every shard sent all of its 4 * tiles maxima
    (driver.hip makes the same decision)."""
    R, B, G = g.shape
    m_total = 256 * tiles * R
    RG = R * 4 * tiles
    if sent is None:
        sent = G
    j = spec_rank(kprime * m_total / max(n_global, 1))
    if j > RG // 2 or (sent < 4 * tiles and j > sent):
        return None
    theta = pool_kth(g.permute(1, 0, 2).reshape(B, R * G), B, qb.B_pad, j)
    hits = (j + j * j / (2.0 * RG)) * n_local / m_total
    return theta, hits


def score_topk_sharded_local(catalog: Catalog, k: int, queries: Optional[torch.Tensor] = None,
                             liked: Optional[Sequence[Sequence[int]]] = None,
                             exclude=None, group: Optional[dist.ProcessGroup] = None,
                             collectives=None, **kw) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-shard exact top-k (the single-GPU path on each shard) + all-gather + merge."""
    return score_topk_sharded_local_finish(score_topk_sharded_local_submit(
        catalog, k, queries=queries, liked=liked, exclude=exclude, group=group,
        collectives=collectives, **kw))


def score_topk_sharded_local_submit(catalog: Catalog, k: int,
                                    queries: Optional[torch.Tensor] = None,
                                    liked: Optional[Sequence[Sequence[int]]] = None,
                                    exclude=None, group: Optional[dist.ProcessGroup] = None,
                                    collectives=None, shared_threshold: bool = True, **kw):
    """Enqueue a batch of score_topk_sharded_local (its screen and the floor all-gather) and
    return without waiting; score_topk_sharded_local_finish completes it (retries, all-gather,
    merge). Every rank must submit and finish its batches in the same order: the collectives
    are issued in program order, so ranks stay in lockstep. shared_threshold: screen every
    shard at one catalog-wide threshold (_shared_theta) when the batch allows it."""
    g = score_topk_sharded_local_stages(catalog, k, queries=queries, liked=liked,
                                        exclude=exclude, group=group, collectives=collectives,
                                        shared_threshold=shared_threshold, **kw)
    next(g)
    next(g)
    return next(g)


def score_topk_sharded_local_stages(catalog: Catalog, k: int,
                                    queries: Optional[torch.Tensor] = None,
                                    liked: Optional[Sequence[Sequence[int]]] = None,
                                    exclude=None, group: Optional[dist.ProcessGroup] = None,
                                    collectives=None, shared_threshold: bool = True, **kw):
    """score_topk_sharded_local_submit in the three stages of search.score_topk_stages; every
    stage ends by STARTING a collective (shared threshold, floor) that the next stage waits
    for. Interleaving two batches -- stage 1 of batch i+1 before stage 3 of batch i, which runs
    before stage 2 of batch i+1 (run_sharded_steps) -- runs each collective under the other
    batch's kernels. The last next() returns the pending batch."""
    coll = collectives if collectives is not None else TorchCollectives(group)
    liked_arg = counts_t = hook = None
    if liked is not None:
        liked_arg, counts_t, hook = _liked_queries(catalog, liked, coll)
    kw.setdefault("t_floor_hook", lambda v, e: _gathered_floor(coll, v, e, k, kw.get("timer")))
    B = int(queries.shape[0]) if queries is not None else len(liked)
    # the shared threshold only serves the wave-merge screen (k' <= MERGE_WAVE_KMAX); decided
    # from rank-invariant sizes (k against the whole catalog): its all-gather is a collective
    kp_glob = kw.get("kprime") or default_kprime(catalog, min(k, catalog.n_global))
    tiles = shared_sample_tiles(catalog.n_global, coll.world, pad_batch(B)) \
        if shared_threshold and kw.get("fuse", True) and kp_glob <= MERGE_WAVE_KMAX else 0
    if tiles:
        timer = kw.get("timer")
        kw.setdefault("theta_hook", lambda qb, kp: _shared_theta(coll, catalog, qb, kp, tiles,
                                                                 timer, kp_glob))
    g = score_topk_stages(catalog, k, queries=queries, liked=liked_arg, exclude=exclude,
                          liked_counts=counts_t, liked_sum_hook=hook, **kw)
    next(g)
    yield
    next(g)
    yield
    yield next(g), coll, k


def score_topk_sharded_local_finish(sub) -> Tuple[torch.Tensor, torch.Tensor]:
    """Complete a submitted batch: its retries (local), the all-gather of the per-shard exact
    top-k and the merge."""
    return score_topk_sharded_local_finish_start(sub)().settle()


class ShardMerged:
    """A merged batch whose packed exchange may still need the full one: ``settle()`` waits for
    the merge's "incomplete" flag (an event) and, when some rank's entries above the floor did
    not fit its packed capacity, all-gathers the full [B, k] lists and merges again (every rank
    sees the same flag, so every rank issues the same collectives). Returns (scores, rows)."""

    def __init__(self, out_s, out_r, flag_host=None, event=None, full=None, coll=None, k=0,
                 timer=None):
        self.out_s, self.out_r = out_s, out_r
        self._flag, self._event, self._full = flag_host, event, full
        self._coll, self._k, self._timer = coll, k, timer

    def settle(self) -> Tuple[torch.Tensor, torch.Tensor]:
        if self._event is not None:
            self._event.synchronize()
            if int(self._flag[0]):
                s, r = self._full
                ws, wr = _gather_start(self._coll, s), _gather_start(self._coll, r)
                gs, gr = ws(), wr()
                fs, fr = merge_topk(gs, gr, self._k)
                self.out_s.copy_(fs)
                self.out_r.copy_(fr)
            self._event = self._full = None
        return self.out_s, self.out_r


def pack_results(s: torch.Tensor, r: torch.Tensor, t_floor: Optional[torch.Tensor], world: int,
                 n_global: int):
    """(send buffer, cap) of ebt_shard_pack: a shard's entries with exact score >= t_floor
    (int32 rows behind per-query starts), or None when the compact form does not apply."""
    lib = _lib.load()
    B, k = s.shape
    cap = int(lib.ebt_shard_pack_cap(B, k, world, n_global))
    if not cap:
        return None
    send = torch.empty(int(lib.ebt_shard_pack_bytes(B, cap)), dtype=torch.uint8, device=s.device)
    call("ebt_shard_pack", ptr(s.contiguous()), ptr(r.contiguous()), B, k, ptr(t_floor), cap,
         ptr(send), stream_of(s.device))
    return send, cap


def merge_packed(recv: torch.Tensor, world: int, B: int, k: int, cap: int):
    """ebt_merge_packed over the all-gathered [R, bytes] packed lists: (scores, rows,
    incomplete) with incomplete a device int32 [1]."""
    dev = recv.device
    out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
    out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
    inc = torch.zeros(1, dtype=torch.int32, device=dev)
    call("ebt_merge_packed", ptr(recv.contiguous()), world, B, k, cap, ptr(out_s), ptr(out_r),
         ptr(inc), stream_of(dev))
    return out_s, out_r, inc


def score_topk_sharded_local_finish_start(sub):
    """score_topk_sharded_local_finish up to STARTING the all-gather of the results; the
    returned callable waits for it, merges and returns a ShardMerged (settle() for the final
    answer). The exchange is the compact one when it applies: each shard's entries above the
    catalog-wide floor (pack_results), one all-gather, merge_packed."""
    pending, coll, k = sub
    s, r = score_topk_finish(pending)
    timer = getattr(pending, "timer", None)
    dev = s.device
    t_floor = getattr(pending, "t_floor", None)
    packed = None
    if t_floor is not None:
        with region(timer, "small", dev):
            packed = pack_results(s, r, t_floor, coll.world, pending.catalog.n_global)
    if packed is None:
        ws, wr = _gather_start(coll, s), _gather_start(coll, r)

        def merge():
            with region(timer, "collective_wait", dev):
                gs, gr = ws(), wr()
            with region(timer, "shard_merge", dev):
                return ShardMerged(*merge_topk(gs, gr, k))
        return merge
    send, cap = packed
    wp = _gather_start(coll, send[None])

    def merge_c():
        with region(timer, "collective_wait", dev):
            g = wp()
        with region(timer, "shard_merge", dev):
            out_s, out_r, inc = merge_packed(g, coll.world, s.shape[0], k, cap)
        flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
        flag.copy_(inc, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        return ShardMerged(out_s, out_r, flag, ev, (s, r), coll, k, timer)
    return merge_c


def run_sharded_steps(make_stages, n: int):
    """Drive n batches through score_topk_sharded_local_stages, two in flight: per step
    [stage 1 of i] [stage 3 of i-1] [stage 2 of i] [finish of i-1 up to its gather]
    [settle of i-3] [merge of i-2]. A merged batch is settled (ShardMerged.settle: its packed
    exchange's completeness flag read) one step later, after a host wait that its merge precedes
    on the stream, so the host never waits for the newest work. make_stages() returns a fresh
    generator; returns the last batch's (scores, rows)."""
    if n < 1:
        return None
    prev = make_stages()
    next(prev)
    next(prev)
    merge_prev, merged = None, None
    for _ in range(1, n):
        cur = make_stages()
        next(cur)                      # stage 1 of i: its threshold gather starts
        sub = next(prev)               # stage 3 of i-1: rescore (its floor gathered meanwhile)
        next(cur)                      # stage 2 of i: screen; its floor gather starts
        merge = score_topk_sharded_local_finish_start(sub)
        if merged is not None:
            merged.settle()
        if merge_prev is not None:
            merged = merge_prev()
        merge_prev, prev = merge, cur
    merge = score_topk_sharded_local_finish_start(next(prev))
    if merged is not None:
        merged.settle()
    if merge_prev is not None:
        merge_prev().settle()
    return merge().settle()


# ------------------------------------------------------------------ the C ABI's sharded step --
class RcclComm:
    """An RCCL communicator owned by libebert (include/ebert.h ebt_rccl_*), for the C ABI's
    row-sharded step: rank 0's unique id travels through the torch.distributed group (any
    backend), every rank then joins with its HIP device current. ``comm(n_global)`` is the
    ebt_comm whose all-gather is the library's own ncclAllGather (no Python per collective)."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None) -> None:
        import ctypes
        lib = _lib.load()
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        uid = ctypes.create_string_buffer(128)
        obj = [None]
        if self.rank == 0:   # a failure here reaches every rank (None), never half of them
            try:
                call("ebt_rccl_unique_id", uid, 128)
                obj = [uid.raw]
            except EbertError:
                obj = [None]
        dist.broadcast_object_list(obj, src=0, group=group)
        if obj[0] is None:
            raise EbertError("ebt_rccl_unique_id failed on rank 0 (RCCL not loadable?)")
        uid = ctypes.create_string_buffer(obj[0], 128)
        h = ctypes.c_void_p()
        call("ebt_rccl_comm_init", uid, self.rank, self.world, ctypes.byref(h))
        self.handle = h.value
        self._fn = ctypes.cast(lib.ebt_rccl_all_gather, _lib.ALLGATHER_FN)
        self._sum = ctypes.cast(lib.ebt_rccl_all_reduce_f64, _lib.ALLREDUCE_F64_FN)

    def comm(self, n_global: int) -> "_lib.EbtComm":
        return _lib.EbtComm(self.rank, self.world, n_global, self._fn, self.handle, self._sum)

    def close(self) -> None:
        if self.handle:
            _lib.load().ebt_rccl_comm_destroy(self.handle)
            self.handle = None


class TorchGatherComm:
    """The same ebt_comm with the all-gather done by a Python callback over torch.distributed
    (gloo on a one-GPU rehearsal, thread-simulated ranks in tests): the library's send / recv
    pointers lie inside tensors registered here (the step's workspaces), which the callback
    views and hands to ``coll.all_gather_into`` (or dist.all_gather_into_tensor)."""

    def __init__(self, rank: int, world: int, group: Optional[dist.ProcessGroup] = None,
                 gather=None) -> None:
        import weakref
        self.rank, self.world, self.group = rank, world, group
        self._gather = gather
        self._bufs = []
        # the C callback holds only a weak reference: a bound method would make a cycle
        # (self -> callback -> self) that keeps the registered workspaces alive until a GC pass
        ref = weakref.ref(self)

        def cb(ctx, send, recv, nbytes, stream):
            me = ref()
            return me._callback(ctx, send, recv, nbytes, stream) if me is not None else -1
        self._fn = _lib.ALLGATHER_FN(cb)
        self.error: Optional[BaseException] = None

    def register(self, t: torch.Tensor) -> None:
        self._bufs.append(t)

    def _view(self, p: int, nbytes: int) -> torch.Tensor:
        for t in self._bufs:
            base = t.data_ptr()
            size = t.numel() * t.element_size()
            if base <= p and p + nbytes <= base + size:
                return t.view(torch.uint8).view(-1)[p - base:p - base + nbytes]
        raise EbertError(f"all-gather buffer {p:#x} (+{nbytes}) is not in a registered tensor")

    def _callback(self, ctx, send, recv, nbytes, stream) -> int:
        try:
            import contextlib
            s = self._view(send, nbytes)
            r = self._view(recv, nbytes * self.world)
            # the library's stream (NULL -- ctypes None -- is the device's default stream)
            ctx = (torch.cuda.stream(torch.cuda.ExternalStream(stream, device=s.device))
                   if stream else contextlib.nullcontext())
            with ctx:
                if self._gather is not None:
                    self._gather(r, s)
                else:
                    dist.all_gather_into_tensor(r, s, group=self.group)
            return 0
        except BaseException as e:  # noqa: BLE001 -- surfaces as EBT_EHIP, kept for the caller
            self.error = e
            return -1

    def comm(self, n_global: int) -> "_lib.EbtComm":
        return _lib.EbtComm(self.rank, self.world, n_global, self._fn, None)

    def close(self) -> None:
        self._bufs = []


class ShardedTopk:
    """ebt_cosine_topk_sharded_submit / _finish / _wait (include/ebert.h) over one rank's shard:
    the whole row-sharded step inside libebert, batches in flight. ``slots`` workspaces (each
    with its host buffer, pending record and outputs) cycle; with the default 3 a caller runs
    per step submit(i), finish(i-1), wait(i-2) (``run``). comm: RcclComm or TorchGatherComm.
    Reference: /root/reference/src/backend/app/lib.py:51-55 per shard, merged across shards."""

    def __init__(self, catalog: Catalog, k: int, B: int, comm, slots: int = 3, timer=None,
                 kprime: Optional[int] = None, fuse: bool = True) -> None:
        import ctypes
        self.catalog, self.k, self.B, self.timer = catalog, k, B, timer
        self._comm_owner = comm
        self.comm = comm.comm(catalog.n_global)
        self.opt = _lib.EbtOptions(kprime=int(kprime or 0),
                                   flags=0 if fuse else _lib.EBT_FLAG_NO_FUSE, chunk_rows=0)
        lib = _lib.load()
        need = lib.ebt_sharded_workspace_bytes(ctypes.byref(catalog.cstruct),
                                               ctypes.byref(self.comm), B, k,
                                               ctypes.byref(self.opt))
        if need == 0:
            raise EbertError(f"ebt_sharded_workspace_bytes: batch {B}, k={k} over this shard "
                             "is not supported")
        dev = catalog.device
        self.ws_bytes = int(need)
        self.ws = [torch.empty(need, dtype=torch.uint8, device=dev) for _ in range(slots)]
        self.host = [torch.zeros(B + 2, dtype=torch.int32, pin_memory=True) for _ in range(slots)]
        self.pend = [_lib.EbtShardedPending() for _ in range(slots)]
        self.out = [(torch.empty((B, k), dtype=torch.float64, device=dev),
                     torch.empty((B, k), dtype=torch.int64, device=dev)) for _ in range(slots)]
        self.keep = [None] * slots
        if isinstance(comm, TorchGatherComm):
            for w in self.ws:
                comm.register(w)
        # the per-call constants of submit (host work per step: every ctypes conversion counts)
        self._fn_submit = lib.ebt_cosine_topk_sharded_submit
        self._fn_finish = lib.ebt_cosine_topk_sharded_finish
        self._fn_wait = lib.ebt_cosine_topk_sharded_wait
        self._cat_ref = ctypes.byref(catalog.cstruct)
        self._comm_ref = ctypes.byref(self.comm)
        self._opt_ref = ctypes.byref(self.opt)
        self._slot_args = [(ptr(self.ws[i]), self.ws_bytes, ptr(self.out[i][0]),
                            ptr(self.out[i][1]), ptr(self.host[i]), ctypes.byref(self.pend[i]))
                           for i in range(slots)]
        self._pend_refs = [ctypes.byref(p) for p in self.pend]
        self._timer_h = timer.handle if timer is not None else None

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            err = getattr(self._comm_owner, "error", None)
            msg = _lib.load().ebt_last_error().decode(errors="replace")
            raise EbertError(f"ebt_cosine_topk_sharded_{what} failed with status {rc}: {msg}"
                             + (f" (all-gather: {err!r})" if err is not None else ""))

    def submit(self, slot: int, queries: Optional[torch.Tensor] = None, liked=None,
               exclude=None) -> None:
        """Enqueue one batch into workspace `slot` (free: its previous batch waited)."""
        import ctypes
        dev = self.catalog.device
        q_ptr, q_dt, ldq, lo, lr = None, 0, 0, None, None
        if queries is not None:
            require = queries.is_cuda and queries.dim() == 2 and queries.shape[0] == self.B
            if not require or queries.stride(1) != 1:
                raise EbertError(f"queries must be a contiguous-row [B={self.B}, d] GPU tensor")
            q_ptr, q_dt, ldq = ptr(queries), _lib.DTYPE_CODE[queries.dtype], queries.stride(0)
        else:
            lo, lr = liked if isinstance(liked, tuple) else csr_from_lists(liked, dev)
        eo = er = None
        if exclude is not None:
            eo, er = exclude if isinstance(exclude, tuple) else csr_from_lists(exclude, dev)
        self.keep[slot] = (queries, lo, lr, eo, er)
        ws, ws_bytes, s, r, host, pend = self._slot_args[slot]
        rc = self._fn_submit(self._cat_ref, self._comm_ref, q_ptr, q_dt, self.B, ldq, ptr(lo),
                             ptr(lr), self.k, ptr(eo), ptr(er), self._opt_ref, ws, ws_bytes, s, r,
                             host, pend, self._timer_h, stream_of(dev))
        if rc:
            self._check(rc, "submit")

    def finish(self, slot: int) -> None:
        rc = self._fn_finish(self._pend_refs[slot])
        if rc:
            self._check(rc, "finish")

    def wait(self, slot: int) -> Tuple[torch.Tensor, torch.Tensor]:
        rc = self._fn_wait(self._pend_refs[slot])
        if rc:
            self._check(rc, "wait")
        self.keep[slot] = None
        return self.out[slot]

    def __call__(self, queries=None, liked=None, exclude=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """One batch, blocking (slot 0)."""
        self.submit(0, queries=queries, liked=liked, exclude=exclude)
        self.finish(0)
        return self.wait(0)

    def run(self, n: int, queries: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """n batches of `queries`, three in flight: per step submit(i), finish(i-1), wait(i-2).
        Returns the last batch's (scores, rows), final."""
        S = len(self.ws)
        if S < 3:
            raise EbertError("run() needs 3 slots (a batch's buffers live until its wait)")
        out = None
        for i in range(n + 2):
            if i < n:
                self.submit(i % S, queries=queries)
            if 1 <= i <= n:
                self.finish((i - 1) % S)
            if i >= 2:
                out = self.wait((i - 2) % S)
        return out
