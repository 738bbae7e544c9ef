#!/usr/bin/env python
"""Split a rocprofv3 kernel trace of one end-to-end PPO iteration (bench.py --e2e-iters 1) into its rollout and its
update: the timed update starts after the last rollout encoder launch, the rollout after the warm-up update; per phase
the kernels by total time, with calls and time per minibatch for the update (the minibatches are counted by the
attn_bwd1 launches).  Diagnostic.

    python tools/e2e_split.py <trace dir or csv> [--top 30]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def short(n):
    if n.startswith("Cijk") and "_MT" in n:
        return n[:24] + ".." + "MT" + n.split("_MT")[1].split("_")[0]
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    path = a.path
    if not path.endswith(".csv"):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows, grids = [], defaultdict(set)
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        grids[short(r["Kernel_Name"])].add(f"{g}/{r.get('Workgroup_Size') or r.get('Workgroup_Size_X') or ''}")
    rows.sort()
    # the timed update: everything after the last rollout encoder launch (bench.py's e2e runs a warm-up update,
    # then the timed rollout and update); the rollout: from the first rollout encoder launch after the warm-up
    t_up = max(s for s, _, n in rows if "attn_pool_x3" in n or "attn_pool_kernel" in n)
    t_up = next(s for s, _, n in rows if s > t_up)
    t_wu = max(s for s, _, n in rows if "attn_bwd2" in n and s < t_up) if any(
        "attn_bwd2" in n and s < t_up for s, _, n in rows) else 0
    nmb = sum(1 for s, _, n in rows if "attn_bwd1" in n and s >= t_up)
    for phase, sel in (("rollout (after the warm-up update)", lambda s: t_wu < s < t_up), ("update", lambda s: s >= t_up)):
        agg = defaultdict(lambda: [0, 0.0])
        span = [None, None]
        for s, e, n in rows:
            if not sel(s):
                continue
            agg[short(n)][0] += 1
            agg[short(n)][1] += (e - s) / 1e6
            span[0] = s if span[0] is None else min(span[0], s)
            span[1] = e if span[1] is None else max(span[1], e)
        tot = sum(v[1] for v in agg.values())
        wall = (span[1] - span[0]) / 1e6 if span[0] is not None else 0.0
        div = nmb if phase == "update" and nmb else 1
        unit = f"per minibatch ({nmb})" if div > 1 else "total"
        print(f"== {phase}: kernels {tot:.2f} ms, wall {wall:.2f} ms; {unit}")
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
            gs = sorted(grids[k])
            print(f"  {k:72s} calls {c / div:7.1f}  ms {t / div:8.3f}  avg_us {1e3 * t / c:9.1f}  grid/wg "
                  f"{' '.join(gs[:3])}{' ...' if len(gs) > 3 else ''}")


if __name__ == "__main__":
    main()
