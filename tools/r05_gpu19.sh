#!/bin/bash
# round-5 GPU check 19: the stores' cache policy re-checked on the final kernels (batched tile store): obs tile
# write-through (QS_WT_OBS, default 1) and the state stores' policy (QS_STATE_AUX: sc1 default, 0 plain, 2 nt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in c3 c2; do
  CONFIG=$c STEPS=2000 timeout -k 10 400 bash tools/ab_jit.sh def: obsplain:-DQS_WT_OBS=0 stplain:-DQS_STATE_AUX=0 stnt:-DQS_STATE_AUX=2 def2: obsplain2:-DQS_WT_OBS=0 stplain2:-DQS_STATE_AUX=0 stnt2:-DQS_STATE_AUX=2 || exit $?
done
