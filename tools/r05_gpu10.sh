#!/bin/bash
# round-5 GPU check 10: scenario kernels bitwise vs round 4 (base headers on the round-5 replay-argument ABI)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise10.log 2>&1 || { tail -5 gpurun_out/r05/scen_bitwise10.log; exit 1; }
grep -E "DIFF|identical" gpurun_out/r05/scen_bitwise10.log | tail -8
MODES="dynamic_formations mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
