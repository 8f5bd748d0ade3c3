"""Is a config's step loop bound by the host? (round 6)

bench.py's N = 1 loop submits batch i+1 (score_topk_submit -> ebt_cosine_topk_submit) before it
finishes batch i (score_topk_finish: the certificate event, then the results). If the host's own
work per step -- Python + ctypes + the C entry's launches -- approaches the GPU's step time, the
GPU waits for the host between batches and the wall time tracks the host, not the kernels.
This times, over the same batches as bench.py:
  * the pipelined loop's wall time per step (what bench.py's `value` is made of);
  * the host time inside submit() and inside finish() per step (perf_counter around each call;
    finish's includes its wait for the event);
  * the GPU-only time per step: the same submits enqueued back to back behind a blocker kernel
    (torch.cuda._sleep) so that no GPU gap depends on the host, measured with hipEvents.

    python tools/host_probe.py --config C2 --steps 200
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--depth", type=int, default=1,
                    help="batches submitted ahead of the one being finished (bench.py: 1)")
    ap.add_argument("--burst", type=int, default=0,
                    help="untimed steps run pipelined (one burst) right before the timed loop")
    ap.add_argument("--timer", action="store_true",
                    help="time the filter GEMM's launches as bench.py does (timer.only)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    ebt.load()
    cat = ebt.Catalog(bench.make_catalog_shard(cfg, 0, cfg["n"], dev))
    q = bench.make_queries(cfg, dev)
    k = cfg["k"]
    torch.cuda.synchronize()

    timer = None
    if a.timer:
        timer = ebt.Timer()
        timer.only("gemm_filter")

    def submit():
        return ebt.score_topk_submit(cat, k, queries=q, timer=timer)

    for _ in range(5):
        ebt.score_topk_finish(submit())
    torch.cuda.synchronize()

    if a.burst:
        prev = None
        for _ in range(a.burst):
            p = submit()
            if prev is not None:
                ebt.score_topk_finish(prev)
            prev = p
        ebt.score_topk_finish(prev)
        torch.cuda.synchronize()

    # 1. the pipelined loop (bench.py's), with the host time of each call
    if timer is not None:
        timer.reset()
    t_sub = t_fin = 0.0
    pending = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s0 = time.perf_counter()
        pending.append(submit())
        s1 = time.perf_counter()
        t_sub += s1 - s0
        if len(pending) > a.depth:
            ebt.score_topk_finish(pending.pop(0))
            t_fin += time.perf_counter() - s1
    for p in pending:
        ebt.score_topk_finish(p)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    filt = timer.query("gemm_filter") if timer is not None else None

    # 2. GPU-only: every submit enqueued behind a long blocker kernel, then the finishes
    n = min(a.steps, 64)
    ps = []
    torch.cuda._sleep(int(2e9))   # ~1 s of spinning: every submit below is queued before it ends
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    for _ in range(n):
        ps.append(submit())
    h_enq = (time.perf_counter() - h0) / n
    e1.record()
    queued_before_blocker_end = not e0.query()
    for p in ps:
        ebt.score_topk_finish(p)
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / n * 1e-3
    print(json.dumps({
        "config": a.config, "steps": a.steps, "depth": a.depth, "burst": a.burst,
        "wall_ms_per_step": round(wall * 1e3, 4),
        "host_submit_ms": round(t_sub / a.steps * 1e3, 4),
        "host_finish_ms_incl_wait": round(t_fin / max(a.steps - a.depth, 1) * 1e3, 4),
        "gpu_only_ms_per_step": round(gpu * 1e3, 4),
        "gpu_only_steps": n,
        "enqueue_ms_per_submit_behind_blocker": round(h_enq * 1e3, 4),
        "all_enqueued_before_the_blocker_ended": bool(queued_before_blocker_end),
        "timer": ("gemm_filter, " + ("markers" if os.environ.get("EBT_TIMER_MARKERS") == "1"
                                      else "events on the dispatch")) if timer else None,
        "filter_ms_per_launch": (round(filt[0] / max(filt[1], 1), 4) if filt else None),
        "filter_launches_per_step": (round(filt[1] / a.steps, 2) if filt else None),
    }), flush=True)


if __name__ == "__main__":
    main()
