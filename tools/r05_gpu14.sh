#!/bin/bash
# round-5 GPU check 14: scenario-kernel priority drop on by default -- bitwise vs round 4, timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise14.log 2>&1 || { tail -5 gpurun_out/r05/scen_bitwise14.log; exit 1; }
grep -E "DIFF|identical" gpurun_out/r05/scen_bitwise14.log | tail -3
for c in c3 c3mix c3mixr; do CONFIG=$c STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh a: b: || exit $?; done
