#!/usr/bin/env python
"""Print the top rows of a rocprofv3 kernel_stats.csv (short kernel names)."""
import csv
import glob
import sys

path = sys.argv[1]
if not path.endswith(".csv"):
    path = sorted(glob.glob(f"{path}/**/*kernel_stats.csv", recursive=True))[-1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in list(csv.DictReader(open(path)))[:n]:
    name = r["Name"]
    if name.startswith("Cijk"):
        name = name[:24] + ".." + "MT" + name.split("_MT")[1].split("_")[0]
    print(f"{name[:80]:80s} calls {r['Calls']:>6} avg_us {float(r['AverageNs']) / 1e3:9.1f} "
          f"tot_ms {float(r['TotalDurationNs']) / 1e6:8.2f}")
