#!/bin/bash
# round-5 GPU check 12: update path -- LDS-staged layer-0 column statistics, weighted column sums, dW for the mean
# path, two-deep dW prefetch: tests, e2e bench, e2e kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder_train.py tests/test_gpu_trainer.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r05/tests12.log 2>&1 || { grep -E "FAIL|Error|passed|failed" gpurun_out/r05/tests12.log | tail -20; exit 1; }
grep -E "worst|fused|w_fp32|relative|passed|failed" gpurun_out/r05/tests12.log | tail -16
timeout -k 10 400 python bench.py --steps 200 --no-cpu-baseline --e2e-iters 3 > gpurun_out/r05/e2e12.log 2>&1 || exit $?
tail -1 gpurun_out/r05/e2e12.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["end_to_end"]; print({k: d[k] for k in ("value", "s_per_iteration", "rollout_s", "update_s", "update_tflops")})'
bash tools/r05_prof_e2e.sh 2>&1 | head -24
