#!/bin/bash
# round-5: kernel trace of one end-to-end PPO iteration with the fused x3 update (where update_s goes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_e2e -o e2e --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-iters 1 > gpurun_out/r05/prof_e2e.log 2>&1 || exit $?
f=$(ls gpurun_out/r05/prof_e2e/*kernel_stats.csv gpurun_out/r05/prof_e2e/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e9:.3f} s over {sum(int(r['Calls']) for r in rows)} calls")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:150]}")
PY
find gpurun_out/r05/prof_e2e -name "*kernel_trace.csv" -delete
