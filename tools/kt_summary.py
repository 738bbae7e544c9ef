"""Summarise rocprofv3 kernel-trace CSVs: per kernel name, count, mean duration, VGPR / SGPR / LDS / scratch."""
import csv
import glob
import os
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        agg = defaultdict(list)
        meta = {}
        for r in rows:
            k = r.get("Kernel_Name", "?")
            agg[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            meta[k] = {c: r.get(c) for c in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                                            "Scratch_Size", "Private_Segment_Size", "Workgroup_Size", "Grid_Size")}
        print(f)
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            v = sorted(v)
            print(f"  {k[:90]:90s} n={len(v):5d} mean={sum(v) / len(v) / 1e3:8.3f}us med={v[len(v) // 2] / 1e3:8.3f}us {meta[k]}")
