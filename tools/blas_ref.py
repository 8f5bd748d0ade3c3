"""hipBLASLt (torch.matmul) TFLOP/s on the screening GEMM shapes, random operands, for comparison
with tools/kernel_bench.py (same timing method)."""
import json
import torch

from kernel_bench import timeit

dev = torch.device("cuda:0")
for (B, N, d, dt) in [(4096, 262144, 1536, torch.float16), (4096, 262144, 1536, torch.bfloat16),
                      (4096, 262144, 768, torch.float16), (4096, 65536, 1536, torch.float16)]:
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn((B, d), generator=g, device=dev).to(dt)
    c = torch.randn((N, d), generator=g, device=dev).to(dt)
    out = torch.empty((N, B), device=dev, dtype=dt)
    ms = timeit(lambda: torch.mm(c, q.T, out=out))
    tf = 2.0 * B * N * d / (ms * 1e-3) / 1e12
    print(json.dumps({"blas": "torch.mm", "B": B, "N": N, "d": d, "dtype": str(dt), "ms": round(ms, 4),
                      "tflops": round(tf, 1), "out": "same dtype as inputs"}), flush=True)
