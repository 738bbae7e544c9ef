"""Summarise a `gpu_check.sh profpol` run (rocprofv3 kernel trace + one MFMA counter pass over the fused
attention-encoder kernels, tools/rollout_prof.py c3) into one JSON for profiles/.

    python tools/summarize_pol.py --out profiles/r04_pol_<tag>.json [--tree <git describe>]

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (the guide's per-SIMD
normalisation); wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES (the fraction of wave-cycles spent waiting on anything).
"""
import argparse
import collections
import csv
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        if "qs::pol::" in n or "Cijk" in n or "tanh" in n:
            out[n] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                      "pct": round(float(r["Percentage"]), 2)}
    return out


def pmc(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in d.items():
        m = {c: sum(x) / len(x) for c, x in v.items()}
        e = {"counters": {c: round(x) for c, x in m.items()}}
        if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            e["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
            e["wait_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        out[k] = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--tree", default=None)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    tree = a.tree or subprocess.run(["git", "-C", ROOT, "describe", "--always", "--dirty"], capture_output=True,
                                    text=True).stdout.strip()
    res = {"command": "bash tools/gpu_check.sh profpol (rocprofv3 --kernel-trace --stats / --pmc "
                      "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE "
                      "-- python tools/rollout_prof.py c3)",
           "tree": tree, "note": a.note,
           "kernels": kernel_stats(os.path.join(a.dir, "profpol_kt", "kt_kernel_stats.csv")),
           "pmc": pmc(os.path.join(a.dir, "profpol_pmc", "p_counter_collection.csv"))}
    log = os.path.join(a.dir, "profpol_kt.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("max |x3"):
                res["x3_vs_fp32"] = line.strip()
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: (v["avg_us"]) for k, v in res["kernels"].items() if "pol::" in k}, indent=1))


if __name__ == "__main__":
    main()
