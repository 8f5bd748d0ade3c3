"""Where a rescore workgroup's cycles go (diagnostic build _abl/libebert_rst.so: tools/abl_build.sh rst
-DEBT_RESCORE_STAMP; rescore.hip rescore_kernel). Run with EBERT_LIB=_abl/libebert_rst.so:

    EBERT_LIB=_abl/libebert_rst.so python tools/rescore_stamp.py [--config C2]

Runs one batch of the bench configuration through ebt.score_topk after a warm-up, with the
stamp buffer set for the last launches: each query's workgroup (wave 0) records the shader
cycles of the query / list load and compaction, pass A (the list's first k rows), s_min and pass
B's list, pass B, and the ordering + write. Prints the mean / p50 / p90 over the queries per phase.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    import bench
    import robot_ebert_amd as ebt
    from robot_ebert_amd import _lib as L
    cfg = dict(bench.CONFIGS[a.config])
    dev = torch.device("cuda:0")
    emb = bench.make_catalog_shard(cfg, 0, cfg["n"], dev)
    cat = ebt.Catalog(emb)
    q = bench.make_queries(cfg, dev)
    for _ in range(3):
        ebt.score_topk(cat, cfg["k"], queries=q)
    torch.cuda.synchronize()
    lib = L.load()
    lib.ebt_debug_rescore_stamps.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(5 * cfg["b"], dtype=torch.int64, device=dev)
    lib.ebt_debug_rescore_stamps(ctypes.c_void_p(buf.data_ptr()))
    ebt.score_topk(cat, cfg["k"], queries=q)
    torch.cuda.synchronize()
    lib.ebt_debug_rescore_stamps(None)
    v = buf.view(-1, 5).double().cpu()
    v = v[v.sum(1) > 0]
    names = ["list_compact", "pass_a", "smin_list_b", "pass_b", "order_write"]
    out = {"config": a.config, "queries": int(v.shape[0])}
    for i, n in enumerate(names):
        col = v[:, i].sort().values
        out[n] = {"mean": round(float(col.mean()), 1), "p50": float(col[len(col) // 2]),
                  "p90": float(col[9 * len(col) // 10])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
