#!/usr/bin/env python
"""Turn rocprofv3 outputs under gpurun_out/ into the committed summaries under profiles/.

    python tools/summarize_prof.py --round 1 --config c3

Inputs (written on the GPU box by tools/gpu_check.sh):
  gpurun_out/prof_kt/*kernel_stats.csv        rocprofv3 --kernel-trace --stats of bench.py
  gpurun_out/prof_fetch/*counter_collection   --pmc FETCH_SIZE pass
  gpurun_out/prof_write/*counter_collection   --pmc WRITE_SIZE pass (separate: TCC slots)
  gpurun_out/prof_sq/*counter_collection      --pmc SQ_* pass
  gpurun_out/prof_flops/*counter_collection   --pmc SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32 ... pass (optional)
  gpurun_out/calib_{fetch,write}/...           tools/calib/fetch_calib (known byte counts)
Outputs:
  profiles/r<NN>_<config>_kernel_stats.csv   (verbatim copy)
  profiles/r<NN>_<config>_pmc.json           per-launch counters + corrected HBM bytes
  profiles/pmc_<config>.json                 latest (read by bench.py for roofline.traffic)
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
CALIB_BYTES = 256 << 20


def counters(pattern, kernel_sub):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(OUT, pattern)):
        for r in csv.DictReader(open(f)):
            if kernel_sub in r["Kernel_Name"]:
                acc[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--kernel", default="step_kernel")
    ap.add_argument("--prefix", default="prof", help="gpurun_out/<prefix>_{kt,fetch,write,sq} (profa for flavor A)")
    ap.add_argument("--read-shape", default=None, help="calibration kernel for the FETCH_SIZE divisor (default by flavor)")
    args = ap.parse_args()
    tag = f"r{args.round:02d}_{args.config}"
    os.makedirs(PROF, exist_ok=True)
    ks = glob.glob(os.path.join(OUT, f"{args.prefix}_kt", "*kernel_stats.csv"))
    stats = {}
    if ks:
        shutil.copy(ks[0], os.path.join(PROF, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(ks[0])):
            if args.kernel + "<" in r["Name"] or args.kernel + "I" in r["Name"]:
                stats = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                         "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
                break

    # calibration: measured / true bytes for each access shape
    calib = {}
    for kind, pat in (("FETCH_SIZE", "calib_fetch/*counter_collection.csv"), ("WRITE_SIZE", "calib_write/*counter_collection.csv")):
        acc = counters(pat, "")
        for (kname, cname), v in acc.items():
            short = kname.split("(")[0].split()[-1]
            if cname == kind:
                calib[f"{short}:{kind}"] = (sorted(v)[len(v) // 2] * 1024.0) / CALIB_BYTES

    import subprocess
    try:   # the tree the profiles were taken on (gpurun snapshots the working tree: dirty = uncommitted edits)
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                              text=True).stdout.strip()
        # dirty = uncommitted edits to tracked files outside profiles/ (the summaries this script writes there)
        dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no", "--", ".",
                                ":(exclude)profiles"], capture_output=True, text=True).stdout.strip()
        head += "-dirty" if dirty else ""
    except OSError:
        head = None
    res = {"kernel": stats.get("name"), "config": args.config, "tree": head, "kernel_trace": stats,
           "calibration_ratio": calib}
    for pat in ("_fetch/*counter_collection.csv", "_write/*counter_collection.csv", "_sq/*counter_collection.csv",
                "_flops/*counter_collection.csv"):
        for (kname, cname), v in counters(args.prefix + pat, args.kernel).items():
            if not (args.kernel + "<" in kname or args.kernel + "I" in kname):
                continue
            res.setdefault("counters_per_launch", {})[cname] = sum(v) / len(v)
            res.setdefault("launches_sampled", {})[cname] = len(v)
    c = res.get("counters_per_launch", {})
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # gfx950: FETCH_SIZE counts 64 B per 128-B request (MI355X_MICROARCH.md §HBM) -> use the ratio
        # measured on the kernel's own state-word load shape when the calibration ran, else x2: flavor B's
        # 4 sub-lanes per drone read four 64-B row segments per instruction (read_sub64, XCD-mapped like the
        # step), flavor A's 2 sub-lanes 128-B segments (read_b32's shape)
        shape = args.read_shape or ("read_b32" if args.kernel.endswith("_a") else "read_sub64<true>")
        fr = calib.get(f"{shape}:FETCH_SIZE")
        wr = calib.get("write_b32:WRITE_SIZE")
        fetch = c["FETCH_SIZE"] * 1024.0 / (fr if fr else 0.5)
        write = c["WRITE_SIZE"] * 1024.0 / (wr if wr else 1.0)
        res["hbm_read_bytes_per_launch"] = fetch
        res["hbm_write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = fetch + write
        res["correction"] = {"fetch_divisor": fr or 0.5, "write_divisor": wr or 1.0,
                             "source": f"tools/calib/fetch_calib {shape}" if fr else "guide x2 (uncalibrated)"}
    if "SQ_WAVES" in c:
        w = c["SQ_WAVES"]
        res["per_wave"] = {k: c[k] / w for k in c if k.startswith("SQ_") and k != "SQ_WAVES"}
    json.dump(res, open(os.path.join(PROF, f"{tag}_pmc.json"), "w"), indent=1)
    json.dump(res, open(os.path.join(PROF, f"pmc_{args.config}.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
