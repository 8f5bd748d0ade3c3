"""Does overlapping batch i's serial tail (the exact rescore) with batch i+1's screen pay on
MI355X? (C3's ~0.9 ms per step after the filter GEMM runs with the GPU
otherwise idle.)

    EBERT_LIB=_abl/libebert_grid.so EBT_QP_GRID=<n> python tools/overlap_probe.py [--tail-cus 2]

The persistent screening GEMM holds every CU's register file and 148 KiB of its LDS, so a kernel
on another stream cannot share a CU with it: overlap needs the CUs split. Two CU-masked streams
(hipExtStreamCreateWithCUMask): the screen's stream gets all but --tail-cus CUs per XCD and the
GEMM's persistent grid is sized to them (ablation build tools/abl_build.sh grid
-DEBT_GRID_OVERRIDE, EBT_QP_GRID = 8 x (32 - tail)); the tail stream gets the rest and runs the
previous batch's rescore. First a probe kernel finds which mask bit is which XCD (reading
HW_REG_XCC_ID), so that the split is the same on every XCD (the GEMM's walk assumes workgroup
b runs on XCD b % 8). Modes, each over --batches C3 batches (4096 queries x 1M x 1536 f32,
top-100), after warm-up:
  serial_full:   query prep + screen + rescore per batch on one unmasked stream (the product's
                 order; the grid override unset);
  serial_masked: the same split into the two masked streams, each batch's rescore waited for
                 before the next screen (the cost of the smaller GEMM grid and of the rescore
                 on the tail CUs, no overlap);
  overlapped:    batch i+1's prep + screen on the GEMM stream while batch i's rescore runs on the
                 tail stream.
One JSON line: ms per batch of each mode, the stage times, and whether the rows equal the serial
answer.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# the probe kernel's code object, built on the CPU beforehand:
#   hipcc --offload-arch=gfx950 --genco tools/hw_probe.hip -o _abl/hw_probe.co
PROBE_CO = os.path.join(ROOT, "_abl", "hw_probe.co")


def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_uint32)]
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return h


def masked_stream(h, bits, dev):
    words = (ctypes.c_uint32 * 8)()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = h.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=dev), s


def xcd_of_bits(h, dev):
    """mask bit -> (XCD, CU, SE), by one probe workgroup per single-bit stream."""
    co = PROBE_CO
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    h.hipModuleLoad.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p]
    h.hipModuleGetFunction.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                       ctypes.c_char_p]
    h.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint] * 6 + [
        ctypes.c_uint, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
    assert h.hipModuleLoad(ctypes.byref(mod), co.encode()) == 0
    assert h.hipModuleGetFunction(ctypes.byref(fn), mod, b"hw_probe") == 0
    out = torch.zeros(2, dtype=torch.int32, device=dev)
    xcd = {}
    for bit in range(256):
        ts, raw = masked_stream(h, [bit], dev)
        p = ctypes.c_void_p(out.data_ptr())
        args = (ctypes.c_void_p * 1)(ctypes.addressof(p))
        out.zero_()
        torch.cuda.synchronize()
        rc = h.hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, raw, args, None)
        assert rc == 0, rc
        h.hipStreamSynchronize(raw)
        v = out.cpu().tolist()
        xcd[bit] = (v[0], (v[1] >> 8) & 15, (v[1] >> 13) & 7)   # XCC, CU, SE
        h.hipStreamDestroy(raw)
    return xcd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tail-cus", type=int, default=2, help="CUs per XCD for the tail stream")
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--b", type=int, default=4096)
    ap.add_argument("--layout", default="probe", choices=["probe", "blocked", "interleaved"],
                    help="mask bit -> XCD: measured by the probe kernel (HW_REG_XCC_ID), or "
                         "assumed: 32 consecutive bits per XCD, or bit i on XCD i %% 8")
    a = ap.parse_args()
    import bench
    import robot_ebert_amd as ebt
    from robot_ebert_amd import _lib
    from robot_ebert_amd.search import plan, prepare_queries, run_screen
    ebt.load()
    dev = torch.device("cuda:0")
    h = hip()
    xcd = xcd_of_bits(h, dev)
    per = {}
    for bit, (x, cu, se) in xcd.items():
        if a.layout == "blocked":
            x = bit // 32
        elif a.layout == "interleaved":
            x = bit % 8
        per.setdefault(x, []).append(bit)
    tail_bits = [b for x in sorted(per) for b in sorted(per[x])[:a.tail_cus]]
    gemm_bits = [b for b in range(256) if b not in set(tail_bits)]
    grid_env = os.environ.get("EBT_QP_GRID")
    cfg = dict(bench.CONFIGS["C3"], n=a.n, b=a.b)
    emb = bench.make_catalog_shard(cfg, 0, cfg["n"], dev)
    cat = ebt.Catalog(emb)
    qs = [bench.make_queries(cfg, dev), bench.make_queries(dict(cfg), dev).flip(0).contiguous()]
    k = cfg["k"]
    kp = plan(cat, cfg["b"], k)["kprime"]
    lib = _lib.load()

    def screen(q):
        qb = prepare_queries(cat, queries=q)
        lv, lr, ovf, eps = run_screen(cat, qb, k, kp)
        return qb, lv, lr, ovf, eps

    def rescore(st):
        qb, lv, lr, ovf, eps = st
        B = qb.B
        out_s = torch.empty((B, k), dtype=torch.float64, device=dev)
        out_r = torch.empty((B, k), dtype=torch.int64, device=dev)
        cert = torch.empty(B, dtype=torch.int32, device=dev)
        _lib.call("ebt_rescore", _lib.ptr(qb.q64), B, cat.d, _lib.ptr(cat.data), cat.dtype_code,
                  cat.ld, _lib.ptr(cat.gnorm), 0, _lib.ptr(lv), _lib.ptr(lr), kp, k, cat.n,
                  _lib.ptr(eps), None, _lib.ptr(out_s), _lib.ptr(out_r), _lib.ptr(cert), None,
                  _lib.stream_of(dev))
        return out_s, out_r, cert

    SA, _ = masked_stream(h, gemm_bits, dev)
    SB, _ = masked_stream(h, tail_bits, dev)

    def run(mode, n):
        A = B_ = None
        if mode != "serial_full":
            A, B_ = SA, SB
        outs, prev, keep = [], None, []   # every batch's screen outputs live to the end
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            q = qs[i % 2]
            if mode == "serial_full":
                outs.append(rescore(screen(q)))
                continue
            with torch.cuda.stream(A):
                st = screen(q)
                ev = torch.cuda.Event()
                ev.record(A)
            keep.append(st)
            if mode == "serial_masked":
                with torch.cuda.stream(B_):
                    B_.wait_event(ev)
                    outs.append(rescore(st))
                torch.cuda.current_stream(dev).wait_stream(B_)
                B_.synchronize()
                continue
            # overlapped: this batch's rescore waits for its screen only; the next screen
            # starts at once on A
            with torch.cuda.stream(B_):
                B_.wait_event(ev)
                outs.append(rescore(st))
            prev = st
        if B_ is not None:
            B_.synchronize()
        if A is not None:
            A.synchronize()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3, outs, prev

    res = {"layout": a.layout, "xcds_seen": len(per),
           "tail_cus_per_xcd": a.tail_cus, "gemm_cus": len(gemm_bits), "tail_cus": len(tail_bits),
           "qp_grid_override": grid_env, "bit_to_xcd_sample": {b: xcd[b] for b in (0, 1, 7, 8, 31, 32)}}
    for mode in ("serial_full", "serial_masked", "overlapped", "serial_full"):
        if mode == "serial_full" and grid_env:
            os.environ.pop("EBT_QP_GRID", None)   # read per launch by the ablation build
        elif grid_env:
            os.environ["EBT_QP_GRID"] = grid_env
        run(mode, 2)  # warm
        ms, outs, _ = run(mode, a.batches)
        key = mode if mode not in res else mode + "_again"
        res[key + "_ms_per_batch"] = round(ms, 3)
        if mode == "serial_full" and "ref" not in res:
            ref = [(o[1][:64].cpu(), o[0][:64].cpu()) for o in outs[:2]]
            res["ref"] = True
        else:
            same = all(torch.equal(outs[i][1][:64].cpu(), ref[i % 2][0]) for i in range(2))
            res[key + "_rows_equal"] = bool(same)
        print(json.dumps({mode: round(ms, 3)}), file=sys.stderr, flush=True)
    res.pop("ref", None)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
