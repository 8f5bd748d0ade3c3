"""Debug: certificate histogram of one ebt_cosine_topk_prepared call at a bench shape (no retries)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd.search import (default_kprime, plan, prepare_queries,  # noqa: E402
                                    run_pipeline)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
dev = torch.device("cuda:0")
cfg = dict(bench.CONFIGS["C3"], n=n)
emb = bench.make_catalog_shard(cfg, 0, n, dev)
cat = ebt.Catalog(emb)
q = bench.make_queries(cfg, dev)
qb = prepare_queries(cat, queries=q)
kp = default_kprime(cat, 100)
print("plan", plan(cat, cfg["b"], 100))
s, r, cert = run_pipeline(cat, qb, 100, kp)
c = cert.cpu()
print("kprime", kp, "cert hist", {v: int((c == v).sum()) for v in (-2, -1, 0, 1)})
bad = torch.nonzero(c != 1).flatten()[:8]
print("bad queries", bad.tolist())
from robot_ebert_amd.search import run_screen  # noqa: E402
lv, lr, ovf, eps = run_screen(cat, qb, 100, kp)
o = ovf.cpu()
print("screen ovf hist", {v: int((o == v).sum()) for v in (0, 1, 2)})
bad = torch.nonzero(o != 0).flatten()[:4]
# exact fp32 scores of the bad queries vs the whole shard: where do T and the list sit?
cn = torch.nn.functional.normalize(emb.float(), dim=1)
for b in bad.tolist():
    sc = torch.nn.functional.normalize(q[b].float(), dim=0) @ cn.T
    top = torch.topk(sc, 1200).values
    nl = int((lv[b] > float("-inf")).sum())
    print(b, "ovf", int(o[b]), "T(100th)", float(top[99]), "200th", float(top[199]),
          "list k-th", float(lv[b, 99]), "list entries", nl, "eps", float(eps[b]),
          "rank of list min", int((sc >= lv[b, nl - 1]).sum()) if nl else -1)
