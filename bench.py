"""Benchmark of the recommend/top-K hot path (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]

One step = one batch of B synthetic Gaussian queries through the whole path (query prep ->
fused MFMA screen (pilot, filtered GEMM segments, merges) -> exact float64 rescore ->
certification; for N > 1 the RCCL all-gather of the per-shard top-k + merge). The catalog (seeded Gaussian,
generated on the GPU in fixed 65536-row blocks so every N sees the same global matrix) is
row-sharded over the N ranks and resident in HBM before timing starts: `scaling` = "strong"
(fixed total work). Rank 0 prints ONE JSON line. The CPU baseline (rank 0, N = 1 only) times the
float64 oracle restatement of lib.py:51-55 -- one sklearn-style cosine_similarity + pandas sort
per query, as the reference does -- on a bounded sample of the same queries, and the same sample
is the parity check.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    "C2": dict(n=100_000, d=768, dtype="bf16", b=1024, k=100),
    "C3": dict(n=1_000_000, d=1536, dtype="f32", b=4096, k=100),
    "C4": dict(n=10_000_000, d=768, dtype="bf16", b=8192, k=100),
    "C5": dict(n=50_000_000, d=1536, dtype="f16", b=16384, k=1000),
}
TORCH_DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
METRIC = "queries/sec + top-K index match, 1M×d=1536 batch=4096, at 1/2/4/8 MI355X"
PEAK_F16_TFLOPS = 2500.0   # MI355X dense bf16/f16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # HBM3E spec
BLOCK_ROWS = 65536


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def make_catalog_shard(cfg, begin: int, end: int, device) -> torch.Tensor:
    """Rows [begin, end) of the global seeded catalog (seed 1 + block id per 65536-row block)."""
    out = torch.empty((end - begin, cfg["d"]), dtype=TORCH_DT[cfg["dtype"]], device=device)
    b0 = begin // BLOCK_ROWS
    b1 = (end - 1) // BLOCK_ROWS
    for blk in range(b0, b1 + 1):
        g = torch.Generator(device=device).manual_seed(1_000_003 * 1 + blk)
        r0 = blk * BLOCK_ROWS
        rows = min(BLOCK_ROWS, cfg["n"] - r0)
        x = torch.randn((rows, cfg["d"]), generator=g, device=device, dtype=torch.float32)
        lo, hi = max(begin, r0), min(end, r0 + rows)
        out[lo - begin:hi - begin] = x[lo - r0:hi - r0].to(out.dtype)
    return out


def make_queries(cfg, device) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(2)
    q = torch.randn((cfg["b"], cfg["d"]), generator=g, device=device, dtype=torch.float32)
    return q.to(TORCH_DT[cfg["dtype"]])


def make_exclusions(cfg, r: int) -> list:
    """Per query, up to r distinct seeded random global rows to exclude (SURVEY section 8d:
    seed 3; the rated movies that lib.py:48 drops from the candidates), sorted."""
    rng = np.random.default_rng(3)
    draw = rng.integers(0, cfg["n"], size=(cfg["b"], r), dtype=np.int64)
    return [np.unique(x) for x in draw]


def host_info() -> dict:
    """The host the CPU baseline ran on: usable cores (affinity), the machine's count, model."""
    try:
        cores = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cores = os.cpu_count() or 1
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": cores, "cpu_count_machine": os.cpu_count(), "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "note": "nproc = CPUs in this process's affinity mask; the GPU box grants a share "
                    "of 16 (OMP_NUM_THREADS), which is what the BLAS threads use"}


def blas_threads() -> int:
    try:
        from threadpoolctl import threadpool_info
        return max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    except Exception:
        return 1


def host_blocks(emb: torch.Tensor, rows: int, block: int = 1 << 17):
    """Row blocks [0, rows) of a device catalog as host float32 arrays (exact for f16 / bf16)."""
    for r0 in range(0, rows, block):
        yield r0, emb[r0:min(rows, r0 + block)].float().cpu().numpy()


# the per-query / batched CPU baselines hold their catalog in float64 on the host: above this
# many rows they run on the first BASE_ROWS_MAX rows and the rate is scaled by rows / n (the
# per-query cost is linear in the catalog rows: one pass over the catalog per query / chunk)
BASE_ROWS_MAX = 1_000_000


def cpu_baseline_and_parity(cfg, blocks, n_all: int, q_gpu: torch.Tensor, s_gpu, r_gpu,
                            budget_s: float, n_parity: int = 0,
                            what: str = "full catalog, streamed in row blocks", exclude=None):
    """CPU baselines and the parity sample.

    (i)  reference-faithful, the value reported: the float64 oracle restatement of lib.py:51-55
         per query, as the reference runs it (cosine_similarity re-normalises the catalog on
         every call, mean, pandas sort_values, [:k]);
    (ii) batched: cosine_similarity(Q_chunk, C) for 64 queries at a time + argpartition top-k
         (oracle.restatement.cosine_topk), reported beside it.
    Both on a bounded sample (about budget_s / 2 seconds each). Parity: n_parity evenly spaced
    queries (128 by default, 32 above BASE_ROWS_MAX rows) against the host float64 oracle over
    the FULL catalog, streamed from the device in row blocks (oracle.restatement.
    cosine_topk_stream): rows bit-exact, |score diff| <= 1e-5.
    blocks(rows) yields (first row, host float32 block) over the first `rows` global rows: the
    resident catalog at N = 1, the catalog regenerated from its seeds on rank 0 at N > 1."""
    import pandas as pd
    from oracle import restatement as R
    rows = min(n_all, BASE_ROWS_MAX)
    scale = rows / n_all
    log(f"copying {rows} catalog rows to host (float64) for the CPU baselines")
    C = np.concatenate([b for _, b in blocks(rows)]).astype(np.float64)
    Q = q_gpu.to(torch.float64).cpu().numpy()
    k = cfg["k"]
    threads = blas_threads()
    sub = "full catalog" if rows == n_all else f"first {rows} of {n_all} rows, rate x {scale:g}"
    # (i) per query
    done, t_total = 0, 0.0
    while done < Q.shape[0] and (t_total < budget_s / 2 or done < 2):
        i = done * 97 % Q.shape[0]
        t0 = time.perf_counter()
        sims = R.cosine_similarity(Q[i:i + 1], C)                  # lib.py:51 (normalises C)
        scores = pd.Series(sims.mean(axis=0))                       # lib.py:52
        scores.sort_values(ascending=False)[:k]                     # lib.py:55
        t_total += time.perf_counter() - t0
        done += 1
        if done & (done - 1) == 0:
            log(f"cpu baseline (i) query {done}: {t_total / done:.3f} s/query")
    # (ii) batched, 64 queries per cosine_similarity call
    nb, t_b = 0, 0.0
    while nb < Q.shape[0] and (t_b < budget_s / 2 or nb == 0):
        t0 = time.perf_counter()
        R.cosine_topk(Q[nb:nb + 64], C, k, chunk=64)
        t_b += time.perf_counter() - t0
        nb += min(64, Q.shape[0] - nb)
        if (nb // 64) & (nb // 64 - 1) == 0:
            log(f"cpu baseline (ii): {nb} queries, {t_b / nb:.4f} s/query")
    del C
    hi = host_info()
    base = {"value": done / t_total * scale, "unit": "queries/s", "cores": int(threads),
            "kind": "port",
            "sample": f"(i) {done} queries, one at a time ({sub}): float64 oracle restatement of "
                      "lib.py:51-55 (cosine_similarity incl. catalog re-normalise per call, mean, "
                      "pandas sort_values, [:k]); numpy elementwise 1 thread, BLAS "
                      f"{threads} threads",
            "seconds": round(t_total, 2),
            "batched": {"value": nb / t_b * scale, "unit": "queries/s", "queries": nb,
                        "seconds": round(t_b, 2),
                        "sample": f"(ii) cosine_similarity(Q_chunk of 64, C) + argpartition "
                                  f"top-k, float64 ({sub}), BLAS {threads} threads"},
            "host": hi,
            "note": "reported baseline, not the target"}
    # parity sample over the full catalog (>= 64 queries per config; 32 at
    # the multi-GPU-sized catalogs, where the host oracle streams 10M-50M rows)
    n_par = n_parity or (128 if n_all <= BASE_ROWS_MAX else 32)
    return base, oracle_parity(k, blocks(n_all), Q, s_gpu, r_gpu, n_par, what, exclude)


def global_blocks(cfg, device, block: int = 1 << 17, rows: int = None):
    """Row blocks of the first `rows` (default all) rows of the WHOLE global catalog as host
    float32 arrays, regenerated on `device` from the same seeds every rank's shard came from
    (N > 1: rank 0 holds only its shard)."""
    n = cfg["n"] if rows is None else min(rows, cfg["n"])
    for r0 in range(0, n, block):
        r1 = min(n, r0 + block)
        yield r0, make_catalog_shard(cfg, r0, r1, device).float().cpu().numpy()


def oracle_parity(k: int, blocks, Q: np.ndarray, s_gpu, r_gpu, n_par: int, what: str,
                  exclude=None):
    """n_par evenly spaced queries of the batch against the host float64 oracle streamed over
    the catalog blocks (oracle.restatement.cosine_topk_stream): rows bit-exact, |ds| <= 1e-5.
    exclude: the batch's per-query excluded rows (the oracle drops them as lib.py:55 does)."""
    from oracle import restatement as R
    n_par = min(Q.shape[0], n_par)
    idx = np.unique(np.linspace(0, Q.shape[0] - 1, n_par).astype(np.int64))
    t0 = time.perf_counter()
    ref_s, ref_r = R.cosine_topk_stream(Q[idx], blocks, k + 1,
                                        exclude=None if exclude is None else
                                        [exclude[i] for i in idx],
                                        workers=min(8, max(1, host_info()["nproc"] // 2)))
    t_par = time.perf_counter() - t0
    g_s = s_gpu[torch.from_numpy(idx).to(s_gpu.device)].cpu().numpy()
    g_r = r_gpu[torch.from_numpy(idx).to(r_gpu.device)].cpu().numpy()
    rows_equal = bool(np.array_equal(ref_r[:, :k], g_r))
    max_diff = float(np.max(np.abs(ref_s[:, :k] - g_s)))
    gap = ref_s[:, k - 1] - ref_s[:, k]
    log(f"parity: {len(idx)} queries in {t_par:.1f} s, rows_equal={rows_equal}")
    hit = None
    if exclude is not None:   # no excluded row may come back
        hit = sum(int(np.isin(g_r[j], exclude[i]).sum()) for j, i in enumerate(idx))
    parity = {"queries_checked": int(len(idx)), "rows_bit_exact": rows_equal,
              "excluded_rows_returned": hit,
              "max_abs_score_diff": max_diff, "tolerance": 1e-5,
              "oracle": "float64 restatement (oracle.restatement.cosine_topk_stream) over the "
                        + what,
              "sample": f"{len(idx)} evenly spaced queries of the batch",
              "boundary_risk_queries": int(np.sum(gap < 1e-6)),
              "min_k_gap": float(np.min(gap)), "seconds": round(t_par, 1)}
    return parity


def pmc_traffic(config: str, world: int):
    """(HBM bytes per launch of the dominant kernel, note) from the committed rocprofv3 PMC
    summary (profiles/pmc_<config>_n<N>.json, FETCH_SIZE*2 + WRITE_SIZE, gfx950 correction
    applied by tools/pmc_summary.py); (None, reason) when no summary exists for this config/N."""
    name = f"pmc_{config}_n{world}.json"
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            v = json.load(f).get("hbm_bytes_per_launch")
        return v, f"profiles/{name}: separate --pmc FETCH_SIZE / WRITE_SIZE passes of this command"
    except (OSError, ValueError):
        why = ("no PMC summary for this config and N: rocprofv3 --pmc runs on the one-GPU box "
               "only (one rank), the driver's multi-GPU runs are not profiled")
        return None, why


def measure_topk(run_steps, timer, dev, steps: int, kprime: int, cfg: dict, es: int) -> dict:
    """north_star's second roofline: the top-K stage that moves bytes on the fused path is the
    exact rescore (rescore_kernel: candidate rows gathered from the resident catalog, float64
    dot products, the (score desc, row asc) order, the certificate). Measured over `steps` extra
    batches AFTER the timed region (its hipEvents would add stream gaps to `value`), on the
    launch stream, with the rows each launch gathers counted inside the kernel
    (ebt_timer_count_rows: one atomic per query). Algorithmic bytes per launch = gathered rows x
    (d x element size + 8 for the row's float64 norm) + B x (k' x 12 list bytes + d x 8 query +
    k x 16 results + 8 eps / certificate)."""
    B, d, k = cfg["b"], cfg["d"], cfg["k"]
    timer.count_rows(True)
    timer.only("rescore")
    timer.reset()
    run_steps(steps)
    torch.cuda.synchronize(dev)
    ms, n = timer.query("rescore")
    rows = timer.rows()
    timer.count_rows(False)
    if n == 0 or ms <= 0:
        return {"kernel": "rescore_kernel", "launches": 0, "note": "no rescore launch recorded"}
    per_rows = rows / n
    byts = per_rows * (d * es + 8) + B * (kprime * 12 + d * 8 + k * 16 + 8)
    avg_ms = ms / n
    gbs = byts / (avg_ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "rescore_kernel", "achieved": round(gbs, 1),
            "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
            "launches": n, "avg_ms": round(avg_ms, 4), "rows_per_launch": round(per_rows, 1),
            "rows_per_query": round(per_rows / B, 2), "bytes_per_launch": round(byts),
            "bytes_formula": "rows x (d x es + 8) + B x (k' x 12 + d x 8 + k x 16 + 8); rows "
                             "counted in the kernel",
            "steps": steps,
            "note": "hipEvents around every rescore launch over extra steps after the timed "
                    "region; rows gathered are random 16-byte-vector row reads over the catalog"}


def pmc_kernel_traffic(config: str, world: int, pattern: str):
    """(HBM bytes per launch, kernel key) of the first kernel whose name contains `pattern` in
    the committed PMC summary of this config / N (tools/prof_summary.py), or (None, None)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}_n{world}.json")
    try:
        with open(path) as f:
            ks = json.load(f).get("kernels", {})
    except (OSError, ValueError):
        return None, None
    for name, v in ks.items():
        if pattern in name:
            return v.get("hbm_bytes_per_launch"), name
    return None, None


def device_f64_check(emb: torch.Tensor, q: torch.Tensor, s, r, nq: int, chunk: int = 1 << 18):
    """Parity at full size without the host oracle (which would need the catalog in float64 on
    the host): nq evenly spaced queries against torch float64 on the device -- the catalog
    upcast chunk by chunk, sklearn's normalise (norms < 10 eps -> 1), top-k by (score desc, row
    asc). Not the oracle; a float64 cross-check of the same arithmetic at the bench's shape."""
    B, k = s.shape
    idx = torch.linspace(0, B - 1, nq, device=q.device).round().long().unique()
    q64 = q[idx].double()
    qn = q64.norm(dim=1, keepdim=True)
    q64 = q64 / torch.where(qn < 10 * torch.finfo(torch.float64).eps, torch.ones_like(qn), qn)
    best_s = torch.full((len(idx), 0), float("-inf"), dtype=torch.float64, device=q.device)
    best_r = torch.empty((len(idx), 0), dtype=torch.int64, device=q.device)
    for c0 in range(0, emb.shape[0], chunk):
        c = emb[c0:c0 + chunk].double()
        g = c.norm(dim=1)
        g = torch.where(g < 10 * torch.finfo(torch.float64).eps, torch.ones_like(g), g)
        sc = (q64 @ c.T) / g
        rows = torch.arange(c0, c0 + c.shape[0], device=q.device).expand(len(idx), -1)
        best_s = torch.cat([best_s, sc], 1)
        best_r = torch.cat([best_r, rows], 1)
        # keep k + 8 per query so that equal scores still sort by row below
        ts, ti = torch.topk(best_s, min(k + 8, best_s.shape[1]), dim=1)
        best_s, best_r = ts, torch.gather(best_r, 1, ti)
        del c, sc
    o = torch.argsort(best_r, dim=1)
    best_s, best_r = torch.gather(best_s, 1, o), torch.gather(best_r, 1, o)
    o = torch.argsort(-best_s, dim=1, stable=True)
    ref_s = torch.gather(best_s, 1, o)[:, :k]
    ref_r = torch.gather(best_r, 1, o)[:, :k]
    got_s, got_r = s[idx].double(), r[idx]
    return {"queries_checked": int(len(idx)),
            "rows_bit_exact": bool(torch.equal(got_r, ref_r)),
            "max_abs_score_diff": float((got_s - ref_s).abs().max()),
            "tolerance": 1e-5,
            "oracle": "torch float64 on the device (catalog upcast per chunk), not the host "
                      "restatement"}


def host_boundary(cat, k, q, timer, steps=12):
    """Untimed for `value`: the same step with the queries handed over in host memory and the
    results copied back (PCIe-inclusive). Overlapped (robot_ebert_amd/hostio.py): batch i+1's
    H2D and batch i's D2H run on a copy stream under batch i / i+1's kernels, batches submitted
    before the previous one is finished, as the resident loop does; also the same steps one at
    a time with the copies in line (`serial_ms_per_step`), the round-5 form."""
    import robot_ebert_amd as ebt
    from robot_ebert_amd.hostio import HostStager, run_pipelined
    dev = q.device
    qh = q.cpu().pin_memory()
    timer.only()
    stager = HostStager(dev)

    def submit(qd):
        return ebt.score_topk_submit(cat, k, queries=qd, timer=timer)

    def finish(p):
        return ebt.score_topk_finish(p)

    def overlapped(n):
        outs = None
        for h in run_pipelined(stager, [qh] * n, submit, finish):
            outs = h
        return outs.result()

    overlapped(2)                                   # warm the pinned pools and the copy stream
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    outs = overlapped(steps)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for _ in range(3):
        qd = qh.to(dev, non_blocking=True)
        s, r = finish(submit(qd))
        (s.to("cpu", non_blocking=True), r.to("cpu", non_blocking=True))
        torch.cuda.synchronize(dev)
    el_serial = (time.perf_counter() - t1) / 3
    return {"ms_per_step": round(1e3 * el, 3), "queries_per_s": round(q.shape[0] / el, 1),
            "serial_ms_per_step": round(1e3 * el_serial, 3),
            "h2d_bytes": qh.numel() * qh.element_size(),
            "d2h_bytes": sum(int(a.nbytes) for a in outs), "steps": steps,
            "note": "queries from pinned host memory, results back to host memory; H2D of the "
                    "next batch and D2H of the previous one on a copy stream under the current "
                    "batch's kernels (hostio.run_pipelined); serial_ms_per_step: one step at a "
                    "time, copies in line; never `value`"}


def stage_breakdown(st: dict, ms_per_step: float, world: int) -> dict:
    """The extra (untimed) step's per-stage GPU time against the timed steps' ms_per_step:
    the sum of the recorded stages and the rest. The stages are disjoint regions of the launch
    stream; the rest is GPU-idle time between them (host work, launch gaps) plus, at N = 1, the
    query prep inside the C ABI (not bracketed there). The timed loop overlaps consecutive
    batches (and at N > 1 their collectives), the extra step runs one batch alone, so the sum
    can exceed ms_per_step."""
    total = sum(v[0] for v in st.values())
    return {"sum_ms": round(total, 4), "ms_per_step": round(ms_per_step, 4),
            "rest_ms": round(ms_per_step - total, 4),
            "stages": "gemm (sample / score GEMM), gemm_filter, merge_select (fused-list merges), "
                      "rescore, select, mask; at N > 1 also prep, small (threshold, floor, "
                      "certificate kernels), collective_wait (stream stalls on the all-gathers), "
                      "shard_merge (ebt_merge_topk)",
            "note": "one extra batch after the timed steps, run alone" +
                    (", collectives not overlapped" if world > 1 else "")}


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv, budget_s: float, grace_s: float = 10.0) -> int:
    """`bench.py --gpus N` without an external launcher: start N child processes of this same
    script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (the
    environment torch.distributed.run would give them). Nothing here has touched the GPU: the
    children are started, never exec'd into. Rank 0's stdout carries the JSON line. Fails fast:
    the first non-zero child status stops the other ranks (they would wait in a collective), and
    so does a run that outlives `budget_s` seconds of wall clock (exit status 124). Stopping =
    SIGTERM to every rank's process group, SIGKILL after `grace_s`."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env, start_new_session=True))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}), rendezvous 127.0.0.1:{port}, "
        f"wall-clock budget {budget_s:.0f} s")

    def stop(live):
        for sig, wait_s in ((signal.SIGTERM, grace_s), (signal.SIGKILL, grace_s)):
            for q in live:
                try:
                    os.killpg(q.pid, sig)
                except ProcessLookupError:
                    pass
            t_end = time.monotonic() + wait_s
            while time.monotonic() < t_end and any(q.poll() is None for q in live):
                time.sleep(0.1)
            live = [q for q in live if q.poll() is None]
            if not live:
                return

    rc = 0
    live = list(procs)
    t_stop = time.monotonic() + budget_s
    while live:
        for p in list(live):
            code = p.poll()
            if code is None or p not in live:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log(f"rank pid {p.pid} exited with {code}: stopping the other ranks")
                stop(live)
                live = [q for q in live if q.poll() is None]
        if live and time.monotonic() > t_stop:
            log(f"error: the ranks are still running after the {budget_s:.0f} s budget "
                f"(a collective that never completes?): stopping pids {[q.pid for q in live]}")
            stop(live)
            return 124
        time.sleep(0.2)
    return rc


def init_group(backend: str, world: int, rank: int, timeout_s: float, device=None):
    """init_process_group with a timeout (rendezvous and every collective after it: a rank that
    never joins a collective makes the others fail with an error instead of hanging), then ONE
    verified all-gather of the rank ids: every rank must see [0, 1, ..., world-1], else exit 4.
    The gathered tensor lives on `device` (RCCL) or the CPU (gloo)."""
    import datetime
    import torch.distributed as dist
    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)
    if dist.get_world_size() != world:
        log(f"error: the {backend} process group has {dist.get_world_size()} ranks, expected "
            f"{world}")
        sys.exit(3)
    dev = device if device is not None else torch.device("cpu")
    mine = torch.tensor([rank], dtype=torch.int64, device=dev)
    got = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(got, mine)
    ids = got.cpu().tolist()
    if ids != list(range(world)):
        log(f"error: rank {rank}: the rank-id all-gather over {backend} returned {ids}, "
            f"expected {list(range(world))}")
        sys.exit(4)
    log(f"rank {rank}: {backend} group of {world} verified (rank-id all-gather {ids})")
    return dist


def arith_labels(cfg: dict) -> dict:
    """The line's `dtype` is the arithmetic of the RESULTS: every returned score is recomputed
    in float64 from the catalog's own values (rescore.hip), as the reference computes in float64
    (constants.py:56, lib.py:51). The MFMA screen's operand type (f16 for f32 / f16 catalogs,
    bf16 for bf16 ones) only picks candidates, certified by a rigorous error bound (DESIGN.md
    section 3), and is named in config.arith / config.screen_operands."""
    ops = "bf16" if cfg["dtype"] == "bf16" else "f16"
    return {
        "dtype": "f64",
        "screen_operands": ops,
        "arith": (f"results f64 (every returned score recomputed in float64 from the catalog's "
                  f"own {cfg['dtype']} values); candidate screen on MFMA with {ops} operands and "
                  "f32 accumulation, certified by a rigorous error bound (DESIGN.md section 3); "
                  "uncertified queries rerun, never approximated"),
    }


def dry_run(args, world: int, rank: int) -> None:
    """--dry-run: the multi-rank protocol of a real run on the CPU (gloo), without the GPU
    path: rendezvous, the world-size check, K barrier-bracketed steps of one small all-gather
    each, max-over-ranks timing, and rank 0's single JSON line (n_gpus, rccl_world_size and
    the ranks that reported). CPU test coverage of the launcher (tests/test_bench_launch.py)."""
    import torch.distributed as dist
    if world > 1:
        init_group("gloo", world, rank, args.collective_timeout)
    got = [rank]
    t = torch.tensor([float(rank)])
    calls = [0]

    def step():
        if world > 1:
            calls[0] += 1
            if rank == args.skip_collective_rank and calls[0] == 1:
                # test hook: this rank leaves out one collective; the others must fail with the
                # collective timeout, and the launcher must stop the job, instead of hanging
                log(f"rank {rank}: skipping a collective (--skip-collective-rank)")
                return t.clone()
            out = torch.empty(world)
            dist.all_gather_into_tensor(out, t)
            return out
        return t.clone()
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    g = t
    for _ in range(args.steps):
        g = step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        got = [int(x) for x in g.tolist()]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "queries/s", "n_gpus": world,
                          "rccl_world_size": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(1e3 * elapsed / max(args.steps, 1), 3),
                          "dry_run": True, "ranks_reported": sorted(got),
                          "backend": "gloo" if world > 1 else None}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of the multi-rank protocol (no GPU work)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity", type=int, default=0,
                    help="queries in the host-oracle parity sample (0 = 128, 32 above 1M rows)")
    ap.add_argument("--device-check", type=int, default=0,
                    help="(N = 1) also check this many queries against torch float64 on the GPU")
    ap.add_argument("--n", type=int, default=None, help="override catalog rows (experiments)")
    ap.add_argument("--b", type=int, default=None, help="override batch (experiments)")
    ap.add_argument("--streams", type=int, default=1,
                    help="(N = 1) HIP streams the consecutive batches alternate over")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on GPU 0, gloo instead of RCCL "
                         "(checks the multi-process sharded path and its parity; not scaling)")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="seconds before a rendezvous or collective that never completes fails "
                         "the rank (init_process_group timeout)")
    ap.add_argument("--launch-timeout", type=float, default=1200.0,
                    help="wall-clock budget of a self-launched N > 1 run; the ranks are stopped "
                         "and the exit status is 124 when it is exceeded")
    ap.add_argument("--sharded-path", default="capi", choices=["capi", "python"],
                    help="N > 1: the C ABI's pipelined sharded step (ebt_cosine_topk_sharded_*, "
                         "RCCL all-gathers inside libebert) or the Python pipeline "
                         "(distributed.run_sharded_steps over torch.distributed)")
    ap.add_argument("--exclude", type=int, default=0,
                    help="(N = 1) exclude up to this many seeded random rows per query (the "
                         "rated movies of lib.py:48 / :55; SURVEY section 8d's variant: 128); "
                         "0 = the BASELINE workload, no exclusions")
    ap.add_argument("--skip-collective-rank", type=int, default=-1,
                    help=argparse.SUPPRESS)   # --dry-run test hook (tests/test_bench_launch.py)
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.n:
        cfg["n"] = args.n
    if args.b:
        cfg["b"] = args.b

    if args.gpus < 1:
        log("error: --gpus must be >= 1")
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: this process only starts the ranks (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world} (launch N ranks for --gpus N)")
        sys.exit(2)
    if args.exclude < 0 or (args.exclude and world > 1):
        log("error: --exclude takes a row count >= 0 and runs at N = 1 only")
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, world, rank)
    dist = None
    if args.share_gpu:
        local_rank = 0
    if world > 1:
        torch.cuda.set_device(local_rank)
        if args.share_gpu:
            dist = init_group("gloo", world, rank, args.collective_timeout)
        else:
            dist = init_group("nccl", world, rank, args.collective_timeout,
                              torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    import robot_ebert_amd as ebt
    from robot_ebert_amd.distributed import (RcclComm, ShardedTopk, TorchGatherComm,
                                             run_sharded_steps, score_topk_sharded_local_stages,
                                             shard_range)
    ebt.load()

    begin, end = shard_range(cfg["n"], rank, world)
    log(f"rank {rank}/{world}: generating catalog rows [{begin}, {end}) x {cfg['d']} {cfg['dtype']}")
    emb = make_catalog_shard(cfg, begin, end, dev)
    cat = ebt.Catalog(emb, row_offset=begin, n_global=cfg["n"])
    q = make_queries(cfg, dev)
    torch.cuda.synchronize(dev)
    timer = ebt.Timer()
    k = cfg["k"]

    # A step is submitted (all of its kernels and collectives enqueued) before the previous
    # step is finished (its certificates checked on the host, retries run): the GPU never waits
    # for the host between batches. Every step is a complete batch through the whole path.
    # N > 1: per-shard exact top-k with the shared threshold and the floor cut, all-gather,
    # merge; two batches in flight so that each collective runs under the other batch's kernels
    # (distributed.run_sharded_steps).
    excl, excl_lists = None, None
    if args.exclude:
        # resident in HBM like the queries: the library's device CSR (segments sorted once, as
        # lib.py:48's rated set arrives from SQL), used as it is on every step; a caller's own
        # unsorted device CSR would add one ebt_sort_exclusions launch per call
        from robot_ebert_amd.search import csr_from_lists
        excl_lists = make_exclusions(cfg, args.exclude)
        excl = csr_from_lists(excl_lists, dev)
        log(f"exclusions: {int(excl[1].numel())} rows over {len(excl_lists)} queries (seed 3)")

    def submit():
        return ebt.score_topk_submit(cat, k, queries=q, exclude=excl, timer=timer)

    def finish(p):
        return ebt.score_topk_finish(p)

    # --streams S (N = 1): consecutive batches go to S HIP streams in turn, so that the next
    # batch's query prep and sample GEMM can start on CUs the current batch's last GEMM round,
    # merge and rescore leave idle (each batch keeps its own workspace and outputs)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                  for _ in range(max(1, args.streams) - 1)]

    # N > 1 through the C ABI: the whole step (threshold, floor, rescore, retries, packed
    # results exchange, merge) inside libebert, three batches in flight; the all-gathers are
    # RCCL's (ebt_rccl_all_gather on the library's own communicator) -- or, on a one-GPU gloo
    # rehearsal, torch.distributed's through a callback
    eng, rccl = None, None
    if world > 1 and args.sharded_path == "capi":
        if args.share_gpu:
            comm = TorchGatherComm(rank, world)
        else:
            try:
                rccl = RcclComm()
            except Exception as e:  # noqa: BLE001 -- same collectives through torch.distributed
                log(f"rank {rank}: libebert's RCCL communicator failed ({e})")
            # every rank takes the same path: one rank without the library's communicator sends
            # them all through torch.distributed (mixed paths would wait on each other forever)
            ok = torch.tensor([1 if rccl is not None else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 1:
                comm = rccl
            else:
                if rccl is not None:
                    rccl.close()
                    rccl = None
                log(f"rank {rank}: all-gathers go through torch.distributed instead")
                comm = TorchGatherComm(rank, world)
        eng = ShardedTopk(cat, k, cfg["b"], comm, timer=timer)

    def run_steps(n, log_every=0):
        if eng is not None:
            return eng.run(n, q)
        if world > 1:
            return run_sharded_steps(
                lambda: score_topk_sharded_local_stages(cat, k, queries=q, timer=timer), n)
        pending, out = None, None
        for i in range(n):
            with torch.cuda.stream(streams[i % len(streams)]):
                p = submit()
            if pending is not None:
                out = finish(pending)
            pending = p
            if log_every and (i + 1) % log_every == 0:
                log(f"step {i + 1}/{n} submitted")
        return finish(pending) if pending is not None else out

    for i in range(args.warmup):
        t0 = time.perf_counter()
        run_steps(1)
        torch.cuda.synchronize(dev)
        log(f"warmup {i + 1}/{args.warmup}: {time.perf_counter() - t0:.3f} s")
    from robot_ebert_amd.search import plan
    pl = plan(cat, cfg["b"], k)
    # inside the timed region only the dominant kernel's launches are bracketed by hipEvents
    # (every recorded stage adds ~5 us of stream gaps); the per-stage breakdown comes from one
    # extra, untimed step below
    dom_stage = "gemm_filter" if pl["fused"] else "gemm"
    timer.reset()
    timer.only(dom_stage)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    s, r = run_steps(args.steps, max(1, args.steps // 5))
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    dom_ms, dom_n = timer.query(dom_stage)
    topk = measure_topk(run_steps, timer, dev, max(1, min(args.steps, 10)), pl["kprime"], cfg,
                        emb.element_size())
    topk["traffic"], tk = pmc_kernel_traffic(args.config, world, "rescore_kernel")
    topk["traffic_note"] = (f"profiles/pmc_{args.config}_n{world}.json ({tk}): FETCH_SIZE x 2 + "
                            "WRITE_SIZE per launch, separate --pmc passes" if tk else
                            "no rescore entry in this config's PMC summary")
    timer.reset()
    timer.only()
    run_steps(1)
    torch.cuda.synchronize(dev)
    from robot_ebert_amd._lib import STAGES
    st = {name: timer.query(name) for name in STAGES}
    host = host_boundary(cat, k, q, timer) if world == 1 else None
    n_local = end - begin
    B, d = cfg["b"], cfg["d"]
    head = pl["head_rows"]
    # the speculative screen filters every row (its sample tiles too); the progressive one the
    # rows after its head
    # (less the speculative screen's lead tiles, whose hits come from the sample's own scores)
    spec = pl.get("spec") or {}
    tail = (n_local - 256 * spec.get("lead", 0) if spec else n_local - head) if pl["fused"] else 0
    # dominant kernel: the fused screening GEMM over the tail rows (else the score-writing GEMM)
    if pl["fused"]:
        dom_name = "screen_gemm_qp2_kernel<filter>"
        dom_flops = 2.0 * B * tail * d * args.steps
    else:
        dom_name = "screen_gemm_qp2_kernel<store>"
        dom_flops = 2.0 * B * n_local * d * args.steps
    achieved = dom_flops / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else None
    all_gemm_ms = st["gemm"][0] + st["gemm_filter"][0]   # the extra step
    all_tf = 2.0 * B * n_local * d / (all_gemm_ms * 1e-3) / 1e12 if all_gemm_ms else None
    value = cfg["b"] * args.steps / elapsed
    traffic, traffic_note = pmc_traffic(args.config, world)
    pl_ms = 1e3 * elapsed / args.steps

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "queries/s",
            "n_gpus": world,
            "rccl_world_size": (dist.get_world_size() if dist is not None and not args.share_gpu
                                else (1 if dist is None else 0)),
            "sharded_path": (args.sharded_path if world > 1 else None),
            "sharded_allgather": (None if world == 1 else
                                  "libebert RCCL (ebt_rccl_all_gather)" if rccl is not None else
                                  "torch.distributed all_gather_into_tensor"),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": arith_labels(cfg)["dtype"],
            "data": "synthetic (seeded Gaussian catalog and queries, generated on device)",
            "config": {
                "workload": f"{args.config}: {cfg['n']} items x d={cfg['d']} {cfg['dtype']} catalog, "
                            f"batch={cfg['b']}, top-{k}",
                "n_items": cfg["n"], "d": cfg["d"], "catalog_dtype": cfg["dtype"], "batch": cfg["b"],
                "k": k, "parallelism": f"catalog row-sharded x{world}" +
                ((", gloo" if args.share_gpu else ", RCCL") +
                 " all-gather of each shard's entries above the catalog-wide floor + merge"
                 if world > 1 else ""),
                "arith": arith_labels(cfg)["arith"],
                "screen_operands": arith_labels(cfg)["screen_operands"],
                "exclusions_per_query": (args.exclude or None),
            },
            "roofline": {
                "bound": "mfma", "kernel": dom_name,
                "achieved": round(achieved, 2) if achieved else None,
                "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_F16_TFLOPS, 4) if achieved else None,
                "traffic": traffic,
                "per_launch": {"launches": dom_n, "avg_ms": round(dom_ms / max(dom_n, 1), 4),
                               "flops": dom_flops / max(dom_n, 1),
                               "flops_formula": "2*B*rows*d per launch (rows = the launch's segment "
                                                "of the fused screen; averaged over the "
                                                "segments)"},
                "all_gemm_tflops": round(all_tf, 2) if all_tf else None,
                "per_n": "rank 0's own launches of the dominant kernel over its shard "
                         "(n_local rows); traffic from the committed PMC summary for this "
                         "config and N (profiles/pmc_<config>_n<N>.json), null when none",
            },
            "roofline_topk": topk,
            "plan": pl,
            "stage_ms_per_step": {name: round(v[0], 4) for name, v in st.items()},
            "stage_breakdown": stage_breakdown(st, pl_ms, world),
            "host_boundary": host,
        }
        out["roofline"]["traffic_note"] = traffic_note
        if args.no_cpu_baseline:
            out["cpu_baseline"] = None
        elif world == 1:
            out["cpu_baseline"], out["parity"] = cpu_baseline_and_parity(
                cfg, lambda rows: host_blocks(emb, rows), emb.shape[0], q, s, r,
                args.cpu_budget, args.parity, exclude=excl_lists)
        else:
            # N > 1: rank 0 holds only its shard; the CPU baselines and the parity sample (the
            # merged global top-k of the last timed batch) run over the WHOLE catalog,
            # regenerated block by block from its seeds on rank 0's GPU
            log("cpu baseline + parity: regenerating the global catalog on rank 0")
            out["cpu_baseline"], out["parity"] = cpu_baseline_and_parity(
                cfg, lambda rows: global_blocks(cfg, dev, rows=rows), cfg["n"], q, s, r,
                args.cpu_budget, args.parity,
                "whole global catalog (every shard), regenerated from its seeds on rank 0 and "
                "streamed in row blocks")
        if args.share_gpu and world > 1:
            out["rehearsal"] = (f"{world} ranks sharing GPU 0 over gloo: the multi-process "
                                "sharded path end to end, NOT a scaling measurement")
        if world == 1 and args.device_check > 0:
            out["device_parity"] = device_f64_check(emb, q, s, r, args.device_check)
        print(json.dumps(out), flush=True)
    if rccl is not None:
        torch.cuda.synchronize(dev)
        rccl.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
