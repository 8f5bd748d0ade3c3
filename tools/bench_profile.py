"""Turn a tools/prof_bench.sh run into the committed evidence under profiles/:
  profiles/<round>_bench_<CFG>_kernel_stats.csv  (rocprofv3 --stats summary of bench.py)
  profiles/pmc_<CFG>_n1.json  (HBM bytes per launch of each screening-GEMM kernel; bench.py's
                               roofline.traffic reads hbm_bytes_per_launch of the dominant one)
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is doubled (gfx950: wide streaming reads are tallied
at half their bytes, MI355X_MICROARCH.md "HBM"); Infinity-Cache hits are included in both.
Usage: python tools/bench_profile.py gpurun_out/prof_C3 C3 r1"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the filter-epilogue screening GEMM (EPI_FILTER = 1), f16 or bf16 image, even or odd K-tiles
DOMINANT_RX = re.compile(r"screen_gemm_qp2_kernel<(true|false), 1")


def per_kernel(path, counter):
    tot, n = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ebt::", "")
            tot[name] += float(r["Counter_Value"])
            n[name].add(r["Dispatch_Id"])
    return {k: (tot[k], len(n[k])) for k in tot}


def main(d, cfg, rnd):
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        dst = os.path.join(ROOT, "profiles", f"{rnd}_bench_{cfg}_kernel_stats.csv")
        shutil.copy(stats[0], dst)
        print("wrote", dst)
    fetch = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    avg_ns = {}
    for f in stats:
        for r in csv.DictReader(open(f)):
            avg_ns[r["Name"].split("(")[0].replace("void ebt::", "")] = float(r["AverageNs"])
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb, fn = fetch.get(k, (0.0, 1))
        wb, wn = write.get(k, (0.0, 1))
        rd = fb * 1024 * 2 / max(fn, 1)
        wr = wb * 1024 / max(wn, 1)
        kernels[k] = {"fetch_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                      "hbm_bytes_per_launch": rd + wr, "launches": fn,
                      "avg_ns": avg_ns.get(k)}
    dom = [k for k in kernels if DOMINANT_RX.match(k)]
    dom = max(dom, key=lambda k: kernels[k]["launches"]) if dom else None
    out = {"config": cfg, "round": rnd, "kernels": kernels,
           "dominant": dom,
           "hbm_bytes_per_launch": kernels.get(dom, {}).get("hbm_bytes_per_launch"),
           "note": "FETCH_SIZE x 2 + WRITE_SIZE (KiB -> bytes), Infinity-Cache hits included; "
                   "collected by tools/prof_bench.sh (separate --pmc passes, kernel filter "
                   "screen_gemm) on the bench.py command of this config"}
    dst = os.path.join(ROOT, "profiles", f"pmc_{cfg}_n1.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", dst)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "C3",
         sys.argv[3] if len(sys.argv) > 3 else "r1")
