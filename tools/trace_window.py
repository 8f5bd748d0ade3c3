"""Per-step kernel time of a repeated step from a rocprofv3 kernel trace (`gpu.sh trace OUT ...`).

The window is the last STEPS steps (or STEPS steps from the --first-th anchor launch), each
starting at a launch of the anchor kernel (regex, e.g.
the sample GEMM 'screen_gemm_qp2_kernel<[^,]*, 2'): per kernel the launches and microseconds per
step, the busy time (union of kernel intervals) and the idle gaps per step.

    python tools/trace_window.py gpurun_out/OUT/run_kernel_trace.csv --anchor 'qp2_kernel<false, 2' --steps 20
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--first", type=int, default=None,
                    help="start at this anchor launch (0-based) instead of the last STEPS steps")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [s for s, _, n in rows if re.search(a.anchor, n)]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} anchor launches")
    if a.first is not None:
        if a.first + a.steps >= len(starts):
            raise SystemExit(f"only {len(starts)} anchor launches")
        t0, t1 = starts[a.first], starts[a.first + a.steps]
    else:
        t0, t1 = starts[-a.steps - 1], starts[-1]   # whole steps: [anchor_i, anchor_{i+1})
    per = defaultdict(lambda: [0, 0.0])
    busy, end = 0, t0
    for s, e, n in rows:
        if s < t0 or s >= t1:
            continue
        k = re.sub(r"\(.*", "", n)[:90]
        per[k][0] += 1
        per[k][1] += (e - s) / 1e3
        if e > end:
            busy += e - max(s, end)
            end = e
    st = a.steps
    out = {
        "trace": a.trace, "anchor": a.anchor, "steps": st,
        "step_us": (t1 - t0) / 1e3 / st, "busy_us_per_step": busy / 1e3 / st,
        "idle_us_per_step": ((t1 - t0) - busy) / 1e3 / st,
        "per_kernel": {k: {"launches_per_step": v[0] / st, "us_per_step": round(v[1] / st, 2)}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
