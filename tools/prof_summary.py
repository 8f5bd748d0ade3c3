"""profiles/pmc_<config>_n1.json from a `tools/gpu.sh prof OUT CONFIG` run: per screening-GEMM
kernel, FETCH_SIZE (its own --pmc pass) x 2 KiB-units and WRITE_SIZE (another pass) KiB -> bytes
per launch (the MI355X guide's HBM/rocprofv3 section: gfx950 FETCH_SIZE counts 2 KiB units here,
WRITE_SIZE KiB; Infinity-Cache hits included), the rocprofv3 average duration from the kernel
trace pass, and the dominant kernel's bytes per launch (bench.py's `roofline.traffic`).

    python tools/prof_summary.py gpurun_out/OUT C3 r4 > profiles/pmc_C3_n1.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        name = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"]
        for disp, v in per.items():
            acc[name[disp]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def short(name):
    n = name.split("(")[0].replace("ebt::", "")
    return n


def main(d, config, rnd):
    fetch, nl = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE")
    write, _ = per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    dur = {}
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]))
    kernels = {}
    for k in fetch:
        s = short(k)
        fb = fetch[k] * 2048.0
        wb = write.get(k, 0.0) * 1024.0
        kernels[s] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                      "hbm_bytes_per_launch": fb + wb, "launches": nl[k],
                      "avg_ns": dur.get(s, (None, 0))[0]}
    dom = max(kernels, key=lambda s: (kernels[s]["avg_ns"] or 0) * kernels[s]["launches"])
    print(json.dumps({"config": config, "round": rnd, "kernels": kernels, "dominant": dom,
                      "hbm_bytes_per_launch": kernels[dom]["hbm_bytes_per_launch"],
                      "note": "FETCH_SIZE x 2 + WRITE_SIZE (KiB -> bytes), Infinity-Cache hits "
                              "included; separate --pmc passes (tools/gpu.sh prof, kernel filter "
                              "screen_gemm) on the bench.py command of this config"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
