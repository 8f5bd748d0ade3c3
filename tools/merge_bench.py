"""ebt_merge_topk (the post-all-gather merge of the sharded path) at the 8-GPU shapes: sorted
lists (the co-rank kernel) against the same lists with one rank's list shuffled per query (the
bitonic network the kernel falls back to), hipEvent-timed on one MI355X.

    python tools/merge_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robot_ebert_amd import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for R, B, k in ((8, 4096, 100), (4, 4096, 100), (2, 4096, 100), (8, 16384, 1000),
                    (8, 8192, 100)):
        s = torch.randn((R, B, k), generator=g, device=dev, dtype=torch.float64)
        s = s.sort(dim=2, descending=True).values
        rows = torch.randperm(R * B * k, generator=g, device=dev).view(R, B, k)
        os_ = torch.empty((B, k), dtype=torch.float64, device=dev)
        or_ = torch.empty((B, k), dtype=torch.int64, device=dev)
        out = {"R": R, "B": B, "k": k}
        for name, ss, rr in (("sorted_corank", s, rows),
                             ("unsorted_bitonic", s.flip(2).contiguous(), rows.flip(2).contiguous())):
            def run():
                L.call("ebt_merge_topk", L.ptr(ss), L.ptr(rr), R, B, k, L.ptr(os_), L.ptr(or_),
                       L.stream_of(dev))
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            out[name + "_ms"] = round(e0.elapsed_time(e1) / 20, 4)
            if name == "sorted_corank":
                ref = (os_.clone(), or_.clone())
            else:
                out["same"] = bool(torch.equal(or_, ref[1]) and torch.equal(os_, ref[0]))
        # cold: the lists freshly written by another kernel and the Infinity Cache flushed (a
        # 512 MiB fill) before each merge, as after a real all-gather; events around the merge only
        flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
        tot = 0.0
        for _ in range(10):
            flush.fill_(1)
            s2, r2 = s.clone(), rows.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.call("ebt_merge_topk", L.ptr(s2), L.ptr(r2), R, B, k, L.ptr(os_), L.ptr(or_),
                   L.stream_of(dev))
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        out["sorted_corank_cold_ms"] = round(tot / 10, 4)
        del flush
        out["bytes_read_MB"] = round(R * B * k * 16 / 1e6, 1)
        out["corank_GBs"] = round(R * B * k * 16 / out["sorted_corank_ms"] / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
