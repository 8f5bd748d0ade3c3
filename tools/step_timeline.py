"""One step's kernel sequence from a rocprofv3 kernel trace (--output-format csv): start offset,
duration and the gap before each kernel, for the last complete step (steps delimited by the
dominant kernel's name appearing after a query-prep kernel).

    python tools/step_timeline.py TRACE_CSV [--marker query_prep] [--steps 2]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="query_prep")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 2:
        raise SystemExit(f"only {len(marks)} steps marked by {a.marker}")
    lo, hi = marks[-a.steps - 2], marks[-2]
    t0 = int(rows[lo]["Start_Timestamp"])
    prev = None
    busy = 0.0
    for r in rows[lo:hi]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        prev = e
        busy += (e - s) / 1e3
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} gap {gap:6.1f}  {name}")
    span = (int(rows[hi]["Start_Timestamp"]) - t0) / 1e3
    print(f"{a.steps} steps: span {span:.1f} us, kernels {busy:.1f} us, per step {span / a.steps:.1f} us")


if __name__ == "__main__":
    main()
