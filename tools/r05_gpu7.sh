#!/bin/bash
# round-5 GPU check 7: buffer / replay arguments as VGPR values (QS_VPTR) -- A/B per config, mix stamps, the GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
for c in c3 c3mix c2 c4 c3mixr; do
  CONFIG=$c STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh vptr: novptr:-DQS_VPTR=0 vptr2: novptr2:-DQS_VPTR=0 || exit $?
done
timeout -k 10 200 python tools/phase_stamps.py c3mix > gpurun_out/r05/stamps7_mix.log 2>&1 || exit $?
sed -n 1,7p gpurun_out/r05/stamps7_mix.log; grep -A5 "forces/impulses" gpurun_out/r05/stamps7_mix.log | head -5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_suite7.log 2>&1; rc=$?
tail -3 gpurun_out/r05/gpu_suite7.log; exit $rc
