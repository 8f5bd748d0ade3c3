"""profiles/pmc_<config>_n1.json from a `tools/gpu.sh prof OUT CONFIG` run: per screening-GEMM
kernel, FETCH_SIZE (its own --pmc pass) x 2 KiB-units and WRITE_SIZE (another pass) KiB -> bytes
per launch (the MI355X guide's HBM/rocprofv3 section: gfx950 FETCH_SIZE counts 2 KiB units here,
WRITE_SIZE KiB; Infinity-Cache hits included), the rocprofv3 average duration from the kernel
trace pass, and the dominant kernel's bytes per launch (bench.py's `roofline.traffic`).

    python tools/prof_summary.py gpurun_out/OUT C3 r4 > profiles/pmc_C3_n1.json

With --window W K --anchor REGEX (round 6) every figure is taken over the bench's TIMED steps
only: the dispatches from the W-th to the (W+K)-th launch of the anchor kernel (the sample GEMM,
one per step), in the trace pass and in each PMC pass alike -- not the warm-up, the top-K
measurement steps, the breakdown step or the host-boundary steps after them. The summary then
also recomputes the bench line's roofline frac from the window's rocprofv3 average (the line's
own flops per launch and peak, from the trace pass's bench JSON, OUT/trace.json) next to the
line's hipEvent frac.
"""
import argparse
import re
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def in_window(ids_names, win):
    """Dispatch ids in the window [W-th anchor, (W+K)-th anchor) of (id, name) pairs."""
    if win is None:
        return None
    first, steps, anchor = win
    anchors = sorted(i for i, n in ids_names if re.search(anchor, n))
    if len(anchors) <= first + steps:
        raise SystemExit(f"only {len(anchors)} anchor dispatches ({anchor})")
    lo, hi = anchors[first], anchors[first + steps]
    return {i for i, _ in ids_names if lo <= i < hi}


def per_kernel(d, counter, win=None):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        name = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        keep = in_window(list(name.items()), win)
        for disp, v in per.items():
            if keep is None or disp in keep:
                acc[name[disp]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def trace_durations(d, win):
    """(avg ns, launches) per kernel over the window, from the trace pass's kernel trace."""
    rows = []
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                         int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    keep = in_window([(i, n) for i, n, _ in rows], win)
    acc = defaultdict(list)
    for i, n, ns in rows:
        if i in keep:
            acc[short(n)].append(ns)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def short(name):
    n = name.split("(")[0].replace("ebt::", "")
    return n


def main(d, config, rnd, win=None):
    fetch, nl = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE", win)
    write, _ = per_kernel(os.path.join(d, "write"), "WRITE_SIZE", win)
    dur = {}
    if win is None:
        for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                dur[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]))
    else:
        dur = trace_durations(d, win)
    kernels = {}
    for k in fetch:
        s = short(k)
        fb = fetch[k] * 2048.0
        wb = write.get(k, 0.0) * 1024.0
        kernels[s] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                      "hbm_bytes_per_launch": fb + wb, "launches": nl[k],
                      "avg_ns": dur.get(s, (None, 0))[0]}
    dom = max(kernels, key=lambda s: (kernels[s]["avg_ns"] or 0) * kernels[s]["launches"])
    out = {"config": config, "round": rnd, "kernels": kernels, "dominant": dom,
           "hbm_bytes_per_launch": kernels[dom]["hbm_bytes_per_launch"],
           "note": "FETCH_SIZE x 2 + WRITE_SIZE (KiB -> bytes), Infinity-Cache hits "
                   "included; separate --pmc passes (tools/gpu.sh prof, kernel filter "
                   "screen_gemm) on the bench.py command of this config"}
    if win is not None:
        out["window"] = {"first_step": win[0], "steps": win[1], "anchor": win[2],
                         "what": "the bench's timed steps only (warm-up and the extra steps "
                                 "after the timed region left out), in every pass"}
        line = None
        try:
            for l in open(os.path.join(d, "trace.json")):
                if l.startswith("{"):
                    line = json.loads(l)
        except OSError:
            pass
        if line is not None:
            rf = line["roofline"]
            flops = rf["per_launch"]["flops"]
            avg = kernels[dom]["avg_ns"]
            frac_w = flops / (avg * 1e-9) / 1e12 / rf["peak"]
            out["roofline_check"] = {
                "line_frac": rf["frac"], "line_avg_ms": rf["per_launch"]["avg_ms"],
                "line_launches": rf["per_launch"]["launches"],
                "window_avg_ms": avg / 1e6, "window_launches": kernels[dom]["launches"],
                "window_frac": round(frac_w, 4), "frac_ratio": round(frac_w / rf["frac"], 4),
                "flops_per_launch": flops, "peak_tflops": rf["peak"],
                "what": "the line's flops per launch / the window's rocprofv3 average "
                        "duration / peak, against the line's hipEvent frac (same run)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("config")
    ap.add_argument("round")
    ap.add_argument("--window", nargs=2, type=int, metavar=("W", "K"))
    ap.add_argument("--anchor", default=r"qp2_kernel<(false|true), 2")
    a = ap.parse_args()
    main(a.out, a.config, a.round,
         (a.window[0], a.window[1], a.anchor) if a.window else None)
