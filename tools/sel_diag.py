"""Streaming select diagnostics (GPU): ebt_select_topk over a 4096 x 1M f32 score matrix against
torch's own row reductions over the same matrix (amax, the stream alone).

    EBERT_LIB=... python tools/sel_diag.py [--n 1000000] [--b 4096] [--kp 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import robot_ebert_amd as ebt  # noqa: E402
from robot_ebert_amd import _lib as L  # noqa: E402
from tools.topk_evidence import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--kp", type=int, default=200)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tag", default=os.environ.get("EBERT_LIB", "ship"))
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    ebt.load()
    st = L.stream_of(dev)
    n, B, kp = a.n, a.b, a.kp
    g = torch.Generator(device=dev).manual_seed(1)
    ld = (n + 63) // 64 * 64 + 64
    S = torch.randn((B, ld), generator=g, device=dev) * (1536 ** -0.5)
    ov = torch.empty((B, kp), device=dev)
    oi = torch.empty((B, kp), dtype=torch.int64, device=dev)
    nb = B * n * 4
    out = {"tag": a.tag, "shape": [B, n], "kprime": kp}
    ms = timeit(lambda: L.call("ebt_select_topk", L.ptr(S), None, ld, B, n, 0, kp, 1, L.ptr(ov),
                               L.ptr(oi), kp, st), a.iters)
    out["select_ms"], out["select_TBps"] = round(ms, 4), round(nb / ms / 1e9, 3)
    V = S[:, :n]
    ms = timeit(lambda: torch.amax(V, dim=1), a.iters)
    out["torch_amax_ms"], out["torch_amax_TBps"] = round(ms, 4), round(nb / ms / 1e9, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
