#!/bin/bash
# round-5 GPU check 6: the scenario floats env-major (bitwise vs round 4, scenario / replay / flavor-A parity, mode
# timings, mix stamps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise6.log 2>&1; rc=$?
grep -E "DIFF|identical" gpurun_out/r05/scen_bitwise6.log | tail -8; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_scen.py tests/test_gpu_replay.py tests/test_gpu_parity_a.py -q --timeout 200 --timeout-method thread > gpurun_out/r05/tests6.log 2>&1; rc=$?
tail -3 gpurun_out/r05/tests6.log; [ $rc -ne 0 ] && exit $rc
MODES="static_diff_goal dynamic_formations ep_rand_bezier mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
CONFIG=c3mixr STEPS=1000 timeout -k 10 200 bash tools/ab_jit.sh base: || exit $?
timeout -k 10 200 python tools/phase_stamps.py c3mix > gpurun_out/r05/stamps6_mix.log 2>&1 || exit $?
sed -n 1,7p gpurun_out/r05/stamps6_mix.log; grep -A5 "forces/impulses" gpurun_out/r05/stamps6_mix.log | head -5
