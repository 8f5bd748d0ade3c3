"""Certificate / overflow statistics of one batch's first pass (which queries a step reruns).
Usage: python tools/cert_stats.py --config C4 --n 1250000"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import search  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--n", type=int, default=None)
args = ap.parse_args()
cfg = dict(bench.CONFIGS[args.config])
if args.n:
    cfg["n"] = args.n
dev = torch.device("cuda", 0)
emb = bench.make_catalog_shard(cfg, 0, cfg["n"], dev)
cat = ebt.Catalog(emb)
q = bench.make_queries(cfg, dev)
k = cfg["k"]
qb = search.prepare_queries(cat, q)
kp = search.default_kprime(cat, k)
pl = search.plan(cat, cfg["b"], k)
lv, lr, ovf, eps = search.run_screen(cat, qb, k, kp)
s, r, cert = search.run_pipeline(cat, qb, k, kp)
torch.cuda.synchronize()
o = ovf[: qb.B].cpu()
c = cert.cpu()
res = {"config": args.config, "n": cfg["n"], "kprime": kp, "plan": pl,
       "ovf": {int(v): int((o == v).sum()) for v in o.unique()},
       "cert": {int(v): int((c == v).sum()) for v in c.unique()},
       "eps_mean": float(eps[: qb.B].mean()),
       "kth_minus_kprime_mean": float((lv[:, k - 1] - lv[:, kp - 1]).mean())}
print(json.dumps(res), flush=True)
# the overflowed queries: hits at the speculative threshold (all rows, and the fullest group)
bad = torch.nonzero(o != 0).flatten().tolist()
if bad and pl.get("spec"):
    sp = pl["spec"]
    pooled = search.sample_maxima(cat, qb, sp["tiles"])
    theta = search.pool_kth(pooled[: qb.B], qb.B, qb.B_pad, sp["rank"])
    g = emb.float().norm(dim=1)
    for b in bad[:4]:
        qv = q[b].float()
        sc = (emb.float() @ qv) / g.clamp_min(1e-30) / qv.norm()
        th = float(theta[b])
        hit = sc >= th - 1e-3
        grp = hit[: (len(hit) // 1024) * 1024].view(-1, 1024).sum(1)
        print(json.dumps({"query": b, "theta": th, "hits_all": int(hit.sum()),
                          "max_group_hits": int(grp.max()), "expected": sp["hits"],
                          "kth": float(lv[b, k - 1]), "kprime_th": float(lv[b, kp - 1])}),
              flush=True)
    # the sample maxima of those queries vs torch (per tile, sorted: the 4 subgroup maxima)
    stride = sp["stride"]
    for b in bad[:2]:
        qv = q[b].float()
        ref = []
        for t in range(sp["tiles"]):
            r0 = t * stride * 256
            sc = (emb[r0:r0 + 256].float() @ qv) / g[r0:r0 + 256].clamp_min(1e-30) / qv.norm()
            ref.append(sc.view(4, 64).max(1).values.sort().values)
        ref = torch.stack(ref)
        got = pooled[b].view(sp["tiles"], 4).sort(1).values
        d = (got - ref).abs()
        print(json.dumps({"query": b, "pool_max_abs_diff": float(d.max()),
                          "tiles_off": int((d.max(1).values > 1e-3).sum()),
                          "ref_top": ref.flatten().sort(descending=True).values[:14].tolist(),
                          "got_top": got.flatten().sort(descending=True).values[:14].tolist()}),
              flush=True)
    # where the rows above theta live: per 65536-row generator block, and in the sampled tiles
    for b in bad[:1]:
        qv = q[b].float()
        sc = (emb.float() @ qv) / g.clamp_min(1e-30) / qv.norm()
        th = float(theta[b])
        hit = (sc >= th).float()
        nb = (len(hit) + 65535) // 65536
        per_block = [int(hit[i * 65536:(i + 1) * 65536].sum()) for i in range(nb)]
        in_sample = sum(int(hit[t * stride * 256:t * stride * 256 + 256].sum())
                        for t in range(sp["tiles"]))
        print(json.dumps({"query": b, "hits_per_block": per_block, "hits_in_sample": in_sample,
                          "sample_rows": 256 * sp["tiles"]}), flush=True)
