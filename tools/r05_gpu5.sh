#!/bin/bash
# round-5 GPU check 5: per-lane formation geometry with JIT-constant index math (bitwise vs round 4, scenario parity,
# mode timings) and where mix's loads phase goes (stamps: record loads early / late / skipped)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise5.log 2>&1; rc=$?
tail -3 gpurun_out/r05/scen_bitwise5.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_scen.py -q --timeout 200 --timeout-method thread > gpurun_out/r05/scen_tests5.log 2>&1; rc=$?
tail -2 gpurun_out/r05/scen_tests5.log; [ $rc -ne 0 ] && exit $rc
MODES="static_diff_goal dynamic_formations dynamic_diff_goal swarm_vs_swarm ep_rand_bezier mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
for v in base:"" late:"-DQS_SCW_LATE=1" skip:"-DQS_SCW_SKIP=1"; do
  tag=${v%%:*}; opt=${v#*:}
  QS_JIT_OPTS="$opt" timeout -k 10 200 python tools/phase_stamps.py c3mix > gpurun_out/r05/stamps5_$tag.log 2>&1 || exit $?
  echo "== $tag"; sed -n 1,7p gpurun_out/r05/stamps5_$tag.log; grep -A5 "forces/impulses" gpurun_out/r05/stamps5_$tag.log | head -5
done
