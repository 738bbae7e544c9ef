#!/bin/bash
# round-5 GPU check 4: column statistics + dW rewrite (tests, e2e), scenario-record load placement A/B, scenario
# sub-phase stamps of dynamic_formations and mix
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder_train.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r05/tests5.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|worst|fused|w_fp32|relative|passed|failed" gpurun_out/r05/tests5.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 200 --no-cpu-baseline --e2e-iters 3 > gpurun_out/r05/e2e_x3b.log 2>&1 || exit $?
tail -1 gpurun_out/r05/e2e_x3b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["end_to_end"]; print({k: d[k] for k in ("value", "s_per_iteration", "rollout_s", "update_s", "update_tflops")})'
CONFIG=c3mix STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh early: late:-DQS_SCW_LATE=1 early2: late2:-DQS_SCW_LATE=1 || exit $?
for spec in "c3mix dynamic_formations" "c3mix"; do
  tag=${spec// /_}
  timeout -k 10 200 python tools/phase_stamps.py $spec > gpurun_out/r05/stamps4_$tag.log 2>&1 || exit $?
  head -22 gpurun_out/r05/stamps4_$tag.log; tail -17 gpurun_out/r05/stamps4_$tag.log
done
