#!/bin/bash
# kernel trace (rocprofv3 --stats) of tools/rollout_prof.py: the policy's torch kernels next to the fused ones
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pol -o run --output-format csv -- \
    python tools/rollout_prof.py ${1:-c3} > gpurun_out/prof_pol.log 2>&1
