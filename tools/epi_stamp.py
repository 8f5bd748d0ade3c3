"""Where a filter launch's cycles go, per wave (diagnostic build _abl/libebert_epi.so:
tools/abl_build.sh epi -DEBT_EPI_STAMP; screen_gemm.hip "EBT_EPI_STAMP").

    python tools/epi_stamp.py [--n 100000] [--b 1024] [--d 768] [--img bf16] [--z 2.73] [--cscale]

After ~`secs` seconds of back-to-back launches of one filter segment (random normalised operands,
threshold z / sqrt(d)), one more launch records, per wave, the shader-clock cycles spent in: the
K-loop, the column test, hit staging, hit processing, and the rest of the epilogue (the
workgroup barrier included), plus the tiles and the tiles with hits in that wave. Prints one JSON
line: the means over the waves of cycles per tile for each phase and their shares.
"""
import argparse
import ctypes
import json
import os
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VP, I32, I64, INT = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int
PHASES = ["kloop", "coltest", "stage", "process", "rest"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=333_334)
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--z", type=float, default=3.0)
    ap.add_argument("--img", default="f16", choices=["f16", "bf16"])
    ap.add_argument("--cscale", action="store_true")
    ap.add_argument("--secs", type=float, default=1.5)
    ap.add_argument("--lib", default=os.path.join(ROOT, "_abl", "libebert_epi.so"))
    a = ap.parse_args()
    lib = ctypes.CDLL(a.lib)
    f = lib.ebt_screen_filter
    f.argtypes = [VP, I64, VP, I64, I32, I32, INT, VP, VP, VP, VP, I64, I32, VP, I64, VP, I64, VP]
    f.restype = INT
    lib.ebt_debug_epi_stamps.argtypes = [VP]
    lib.ebt_last_error.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    B, N, d = a.b, a.n, a.d
    g = torch.Generator(device=dev).manual_seed(0)
    dt = torch.float16 if a.img == "f16" else torch.bfloat16
    q = torch.randn((B, d), generator=g, device=dev)
    q = (q / q.norm(dim=1, keepdim=True)).to(dt)
    c = torch.randn((N, d), generator=g, device=dev)
    c = (c / c.norm(dim=1, keepdim=True)).to(dt)
    idt = 2 if a.img == "f16" else 1
    qs = torch.ones(B, device=dev)
    cs = torch.ones(N, device=dev) if a.cscale else None
    G, slots = 256, 32
    groups = (N + G - 1) // G
    cand = torch.empty((B, groups * slots), dtype=torch.int64, device=dev)
    counts = torch.empty((B, groups), dtype=torch.uint8, device=dev)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    thr = torch.full((B,), a.z / d ** 0.5, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731

    def launch():
        rc = f(P(q), B, P(c), N, d, d, idt, P(qs), P(cs), P(thr), P(cand), groups * slots, slots,
               P(counts), groups, P(ovf), 0, st)
        if rc:
            raise RuntimeError(lib.ebt_last_error().decode())
    lib.ebt_debug_epi_stamps(None)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.secs:
        for _ in range(10):
            launch()
        torch.cuda.synchronize()
    buf = torch.zeros(4096 * 8 * 8, dtype=torch.int64, device=dev)
    lib.ebt_debug_epi_stamps(P(buf))
    launch()
    torch.cuda.synchronize()
    lib.ebt_debug_epi_stamps(None)
    v = buf.view(-1, 8).cpu().double()
    v = v[v[:, 5] > 0]
    tiles = v[:, 5]
    per_tile = {ph: float((v[:, i] / tiles).mean()) for i, ph in enumerate(PHASES)}
    tot = sum(per_tile.values())
    hit_tiles = float((v[:, 6] / tiles).mean())
    print(json.dumps({
        "shape": [B, N, d], "img": a.img, "row_scales": bool(a.cscale), "z": a.z,
        "waves": int(v.shape[0]), "tiles_per_wave": float(tiles.mean()),
        "frac_tiles_with_hits_per_wave": round(hit_tiles, 3),
        "hits_per_query": round(float(counts.float().sum(1).mean()), 1),
        "cycles_per_tile": {k: round(x, 1) for k, x in per_tile.items()},
        "share": {k: round(x / tot, 4) for k, x in per_tile.items()}}), flush=True)


if __name__ == "__main__":
    main()
