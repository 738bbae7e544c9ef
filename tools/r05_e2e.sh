#!/bin/bash
# round-5: the fused update's tests, then the end-to-end PPO iteration with the fused x3 update vs torch fp32
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder_train.py tests/test_gpu_trainer.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r05/tests4.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|worst|fused|w_fp32|relative|passed|failed" gpurun_out/r05/tests4.log | tail -40; [ $rc -gt 1 ] && exit $rc
for up in x3 fp32; do
  timeout -k 10 400 python bench.py --steps 200 --no-cpu-baseline --e2e-iters 3 --e2e-update-precision $up > gpurun_out/r05/e2e_$up.log 2>&1 || exit $?
  tail -1 gpurun_out/r05/e2e_$up.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get("end_to_end")))'
done
