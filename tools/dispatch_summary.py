#!/usr/bin/env python
"""Per-dispatch view of a rocprofv3 --kernel-trace CSV: every launch of the kernels matching a pattern, in start
order, with its duration and the idle gap since the previous matching launch ended; plus the launches above
`--outlier` x the mean (index, duration) -- e.g. the driver window's 25 post-reset steps, or c3mix's slow launch.

    python tools/dispatch_summary.py <trace dir or csv> [--match step_kernel] [--outlier 3] [--all]
"""
import argparse
import csv
import glob
import os


def load(path, match):
    if not path.endswith(".csv"):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = [r for r in csv.DictReader(open(path)) if match in r.get("Kernel_Name", "")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="step_kernel")
    ap.add_argument("--outlier", type=float, default=3.0)
    ap.add_argument("--all", action="store_true", help="print every launch (default: the first 40 and the last 5)")
    a = ap.parse_args()
    L = load(a.path, a.match)
    if not L:
        print("no matching launches")
        return 1
    durs = [(e - s) / 1e3 for s, e, _ in L]
    mean = sum(durs) / len(durs)
    print(f"{len(L)} launches of '{a.match}', mean {mean:.3f} us, min {min(durs):.3f}, max {max(durs):.3f}")
    for i, (s, e, n) in enumerate(L):
        if a.all or i < 40 or i >= len(L) - 5:
            gap = (s - L[i - 1][1]) / 1e3 if i else 0.0
            print(f"  #{i:5d} dur {durs[i]:8.3f} us  gap {gap:8.3f} us  {n[:60]}")
    out = [(i, d) for i, d in enumerate(durs) if d > a.outlier * mean]
    print(f"outliers (> {a.outlier} x mean): {len(out)}", [(i, round(d, 1)) for i, d in out[:20]])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
