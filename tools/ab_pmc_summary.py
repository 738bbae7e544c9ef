#!/usr/bin/env python
"""Per-wave SQ counters of qs::step_kernel for every gpurun_out/ab_pmc/<config>_<tag> pass (tools/ab_pmc.sh)."""
import collections
import csv
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
        "SQ_WAVE_CYCLES"]
print(f"{'variant':24s} " + " ".join(f"{k[3:]:>14s}" for k in KEYS))
for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "ab_pmc", "*"))):
    if not os.path.isdir(d):
        continue
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not acc.get("SQ_WAVES"):
        continue
    w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"])
    row = [sum(acc[k]) / len(acc[k]) / w if acc.get(k) else float("nan") for k in KEYS]
    print(f"{os.path.basename(d):24s} " + " ".join(f"{v:14.1f}" for v in row))
