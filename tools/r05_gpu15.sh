#!/bin/bash
# round-5 GPU check 15: the younger-wave priority (mark 11) on / off on the final kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in c3 c2 c4; do
  CONFIG=$c STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh on: off:-DQS_PRIO_AT=-1 on2: off2:-DQS_PRIO_AT=-1 || exit $?
done
