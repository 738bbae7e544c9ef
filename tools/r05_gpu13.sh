#!/bin/bash
# round-5 GPU check 13: C2 phase stamps; the younger wave's priority dropped again at marks 21 / 22 / 23 (C3, c3mix)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 200 python tools/phase_stamps.py c2 > gpurun_out/r05/stamps_c2.log 2>&1 || exit 1
head -14 gpurun_out/r05/stamps_c2.log
for c in c3 c3mix; do
  CONFIG=$c STEPS=2000 timeout -k 10 400 bash tools/ab_jit.sh keep: end21:-DQS_PRIO_END=21 end22:-DQS_PRIO_END=22 end23:-DQS_PRIO_END=23 keep2: end21b:-DQS_PRIO_END=21 end22b:-DQS_PRIO_END=22 end23b:-DQS_PRIO_END=23 || exit $?
done
