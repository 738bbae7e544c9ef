#!/bin/bash
# sub-lanes per drone (QS_QB) A/B of the flavor-B step kernel on CONFIG (kernel us per step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q_ab
CONFIG=${CONFIG:-c3}
for q in ${QS:-1 2 4}; do
  QS_QB=$q timeout -k 10 200 python bench.py --config $CONFIG --steps 2000 --no-cpu-baseline --e2e-iters 0 > gpurun_out/q_ab/${CONFIG}_q$q.log 2>&1 || exit 1
  echo "$CONFIG Q=$q $(tail -1 gpurun_out/q_ab/${CONFIG}_q$q.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"])')"
done
