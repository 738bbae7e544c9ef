#!/bin/bash
# round-5 GPU check 8: the replay arguments through a device pointer (fewer SGPRs, no serialised kernarg loads) --
# timings per config against check 7's, mix stamps, replay / parity tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
for c in c3 c3mix c2 c4 c3mixr; do
  CONFIG=$c STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh rargs: rargs2: || exit $?
done
timeout -k 10 200 python tools/phase_stamps.py c3mix > gpurun_out/r05/stamps8_mix.log 2>&1 || exit $?
sed -n 1,7p gpurun_out/r05/stamps8_mix.log; grep -A5 "forces/impulses" gpurun_out/r05/stamps8_mix.log | head -5
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_parity.py tests/test_gpu_parity_scen.py tests/test_gpu_infos.py -q --timeout 200 --timeout-method thread > gpurun_out/r05/tests8.log 2>&1; rc=$?
tail -3 gpurun_out/r05/tests8.log; exit $rc
