"""Summarise a tools/prof_gemm.sh run: per-dispatch averages of every counter over the screening
GEMM dispatches, plus derived clock / MFMA utilisation / HBM bytes (FETCH_SIZE x 2 KiB-unit
correction of the MI355X guide). Usage: python tools/pmc_summary.py gpurun_out/pmc_NAME [REGEX]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(d, rx="screen_gemm"):
    acc = defaultdict(list)
    kname = None
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            if not re.search(rx, r["Kernel_Name"]):
                continue
            kname = r["Kernel_Name"]
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for disp in per.values():
            for c, v in disp.items():
                acc[c].append(v)
    out = {c: sum(v) / len(v) for c, v in acc.items()}
    dur = None
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if re.search(rx, r["Name"]):
                dur = float(r["AverageNs"])
    out["kernel"] = kname
    out["avg_ns"] = dur
    if dur and "GRBM_GUI_ACTIVE" in out:
        out["clock_GHz"] = out["GRBM_GUI_ACTIVE"] / 8 / dur
    if "SQ_VALU_MFMA_BUSY_CYCLES" in out and "GRBM_GUI_ACTIVE" in out:
        out["mfma_util"] = out["SQ_VALU_MFMA_BUSY_CYCLES"] / (out["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "FETCH_SIZE" in out:
        out["FETCH_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    if "SQ_WAVE_CYCLES" in out:
        w = out["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in out:
                out[c + "_frac"] = out[c] / w
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
