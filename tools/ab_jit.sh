#!/bin/bash
# A/B of specialised-kernel variants on the GPU box: each argument "tag:-DMACRO[,-DMACRO2]" (or "tag:" for
# the baseline) runs bench.py with QS_JIT_OPTS set to the macros.  CONFIG / STEPS from the environment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_jit
CONFIG=${CONFIG:-c3}
STEPS=${STEPS:-2000}
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}; defs=${defs//,/ }
  timeout -k 10 200 env QS_JIT_OPTS="$defs" python bench.py --config $CONFIG --steps $STEPS --no-cpu-baseline \
      --e2e-iters 0 > gpurun_out/ab_jit/${CONFIG}_$tag.log 2>&1
  rc=$?
  echo "$CONFIG $tag rc=$rc $(tail -1 gpurun_out/ab_jit/${CONFIG}_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"], d["value"])' 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
