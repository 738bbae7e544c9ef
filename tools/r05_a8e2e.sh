#!/bin/bash
# round-5: flavor-A end to end (sb_train settings, n_steps 64 for time) with the fused update vs torch fp32
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
for up in x3 fp32; do
  timeout -k 10 500 python bench.py --config a8 --steps 100 --no-cpu-baseline --e2e-iters 1 --e2e-steps 64 --e2e-update-precision $up > gpurun_out/r05/a8_e2e_$up.log 2>&1 || { tail -3 gpurun_out/r05/a8_e2e_$up.log; exit 1; }
  tail -1 gpurun_out/r05/a8_e2e_$up.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["end_to_end"]; print({k: d.get(k) for k in ("value", "s_per_iteration", "rollout_s", "update_s", "update_tflops", "update_precision")})'
done
