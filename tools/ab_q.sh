#!/bin/bash
# A/B of the step kernels' sub-lanes per drone (QS_QB flavor B, QS_QA flavor A) on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_q
run() {  # tag env... -- bench args
  local tag=$1; shift
  timeout -k 10 200 env "$@" > gpurun_out/ab_q/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/ab_q/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"], d["value"])' 2>/dev/null)"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
B="python bench.py --steps 2000 --no-cpu-baseline --e2e-iters 0"
for cfg in c3 c4 c2 c5 c3mix; do
  for q in 4 2 1; do run ${cfg}_qb$q QS_QB=$q $B --config $cfg; done
done
for q in 2 1 4; do run a8_qa$q QS_QA=$q $B --config a8 --steps 1000; done
