"""CPU, world_size 2 (gloo): the multi-GPU plumbing of robot_ebert_amd.distributed.

The GPU kernels cannot run here, so the per-shard top-k comes from the float64 oracle (test
infrastructure); what is exercised is the product's shard partitioning, row offsets, the
all-gather of partial results (`gather_partials`, the same call that runs over RCCL on MI355X)
and the liked-query all-reduce, with the merge checked against the unsharded oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from inputs import COS_CASES, cos_case_inputs


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _body(rank, world, q)
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _body(rank, world, q):
    if True:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        sys.path.insert(0, os.path.join(root, "tests", "golden"))
        from oracle import restatement as R
        from robot_ebert_amd.distributed import gather_partials, shard_range, split_liked

        case = COS_CASES["d768_f32_k100"]
        qv, c, _ = cos_case_inputs(case)
        k = case["k"]
        a, b = shard_range(c.shape[0], rank, world)
        s, r = R.cosine_topk(qv, c[a:b], k)          # this shard's top-k (local rows)
        r = np.where(r >= 0, r + a, -1)                # -> global rows (row_offset)
        gs, gr = gather_partials(torch.from_numpy(s), torch.from_numpy(r))
        ms, mr = R.merge_topk(gs.numpy(), gr.numpy(), k)
        s_full, r_full = R.cosine_topk(qv, c, k)
        ok = bool(np.array_equal(mr, r_full)) and bool(np.allclose(ms, s_full, atol=1e-15))
        # liked-query all-reduce: per-shard sums of normalised liked rows complete the mean
        liked = [[1, 2, 3000, 4000], [5, 4090]]
        local, counts = split_liked(liked, a, b)
        cn = R.normalize_rows(c)
        part = torch.tensor(np.stack([cn[l].sum(0) if l else np.zeros(c.shape[1]) for l in local]))
        dist.all_reduce(part, op=dist.ReduceOp.SUM)
        qmean = part.numpy() / np.array(counts)[:, None]
        want = np.stack([R.mean_cosine_query(c[l]) for l in liked])
        ok = ok and bool(np.allclose(qmean, want, atol=1e-14))
        # the two-phase path's collectives wrapper (the GPU kernels around it need a GPU)
        from robot_ebert_amd.distributed import TorchCollectives
        coll = TorchCollectives()
        g = coll.all_gather(torch.full((3, 4), float(rank)))
        ok = ok and g.shape == (world, 3, 4) and all(bool((g[r] == r).all()) for r in range(world))
        t = torch.full((5,), rank + 1.0, dtype=torch.float64)
        ok = ok and bool((coll.all_reduce_sum(t) == sum(range(1, world + 1))).all())
        m = torch.tensor([rank, 1 - rank], dtype=torch.int32)
        ok = ok and coll.all_reduce_max(m).tolist() == [world - 1, 1]
        # asynchronous all-gathers (the staged per-shard path): started in program order on
        # every rank, completed later, in any order
        w1 = coll.all_gather_start(torch.full((2, 3), float(rank)))
        w2 = coll.all_gather_start(torch.full((4,), 10.0 + rank))
        g2, g1 = w2(), w1()
        ok = ok and g1.shape == (world, 2, 3) and all(bool((g1[r] == r).all())
                                                       for r in range(world))
        ok = ok and g2.shape == (world, 4) and all(bool((g2[r] == 10 + r).all())
                                                    for r in range(world))
        # the per-shard path's global cut: union_floor of the gathered (approx, eps) lists is a
        # lower bound of the global k-th exact score, and no shard cuts a global top-k row
        from floor_ref import union_floor_torch as union_floor
        vals = torch.from_numpy(np.nan_to_num(s, nan=-np.inf).astype(np.float32))
        eps = torch.full((vals.shape[0],), 1e-6, dtype=torch.float32)
        floor = union_floor(coll.all_gather(vals), coll.all_gather(eps), k).numpy()
        ok = ok and bool((floor <= s_full[:, k - 1]).all())
        cut = floor - 1e-6
        for bq in range(vals.shape[0]):
            mine = [int(x) for x in r_full[bq] if a <= x < b]
            kept = set(int(x) for x, v in zip(r[bq], vals[bq].tolist()) if v >= cut[bq])
            ok = ok and set(mine) <= kept
        # and it is tight: about k/world + ties of each shard's k rows survive
        ok = ok and float(np.mean([(vals[bq].numpy() >= cut[bq]).sum()
                                   for bq in range(vals.shape[0])])) < 0.75 * k
        q.put((rank, ok))


def test_sharded_gather_merge_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]
