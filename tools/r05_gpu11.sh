#!/bin/bash
# round-5 GPU check 11: single-drone envs (C2) with 8 sub-lanes per drone (2 waves per SIMD) -- bitwise vs 4, timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
for q in 4 8; do
  QS_QB=$q timeout -k 10 120 python tools/bitwise_ab.py c2 200 > gpurun_out/r05/c2_dig_q$q.log 2>&1 || { tail -3 gpurun_out/r05/c2_dig_q$q.log; exit 1; }
  echo "q$q $(tail -1 gpurun_out/r05/c2_dig_q$q.log)"
done
for r in 1 2; do
  for q in 4 8; do
    QS_QB=$q timeout -k 10 200 python bench.py --config c2 --steps 2000 --no-cpu-baseline --e2e-iters 0 > gpurun_out/r05/c2_q${q}_$r.log 2>&1 || exit $?
    echo "c2 q$q $(tail -1 gpurun_out/r05/c2_q${q}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"], d["value"])')"
  done
done
