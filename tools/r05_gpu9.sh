#!/bin/bash
# round-5 GPU check 9: integer grid dims + branch-free centring sums (bitwise vs round 4, scenario tests, timings,
# stamps of dynamic_formations and mix)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise9.log 2>&1; rc=$?
grep -E "DIFF|identical" gpurun_out/r05/scen_bitwise9.log | tail -8; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_scen.py -q --timeout 200 --timeout-method thread > gpurun_out/r05/scen_tests9.log 2>&1; rc=$?
tail -2 gpurun_out/r05/scen_tests9.log; [ $rc -ne 0 ] && exit $rc
MODES="static_diff_goal dynamic_formations ep_rand_bezier mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
CONFIG=c3mix STEPS=2000 timeout -k 10 200 bash tools/ab_jit.sh a: b: || exit $?
for spec in "c3mix dynamic_formations" "c3mix"; do
  tag=${spec// /_}
  timeout -k 10 200 python tools/phase_stamps.py $spec > gpurun_out/r05/stamps9_$tag.log 2>&1 || exit $?
  echo "== $tag"; sed -n 1,7p gpurun_out/r05/stamps9_$tag.log; grep -A5 "forces/impulses" gpurun_out/r05/stamps9_$tag.log | head -5
done
