#!/bin/bash
# Per-goal-scenario step time of the C3 swarm (c3mix's modes one at a time), plus c3mix PMC passes with the
# instruction-cache and flat-access counters.  GPU box; every step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/r05/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/r05/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"], d["value"])' 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi; }
for m in ${MODES:-static_same_goal static_diff_goal ep_lissajous3D ep_rand_bezier dynamic_same_goal dynamic_diff_goal dynamic_formations swap_goals swarm_vs_swarm mix}; do
  run mode_$m 200 python bench.py --config c3mix --quads-mode $m --steps 1000 --no-cpu-baseline --e2e-iters 0
done
if [ "${PMC:-1}" = 1 ]; then
for c in c3mix c3; do
  run pmc_ic_$c 120 timeout -s KILL 100 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_FLAT SQ_INSTS_FLAT_LDS_ONLY SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY -d gpurun_out/r05/pmc_ic_$c -o p --output-format csv -- python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --graph 0 --e2e-iters 0
done
rm -f gpurun_out/r05/pmc_*/*kernel_trace.csv gpurun_out/r05/pmc_*/*/*kernel_trace.csv
fi
