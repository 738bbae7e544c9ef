#!/bin/bash
# round-5 GPU check: scenario kernels bitwise vs the round-4 kernels, pair rounds bitwise vs the one-pair loop,
# per-mode timing and the C3 rounds A/B, then the new GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise.log 2>&1; rc=$?
tail -28 gpurun_out/r05/scen_bitwise.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/pair_bitwise.py 6 > gpurun_out/r05/pair_bitwise.log 2>&1; rc=$?
cat gpurun_out/r05/pair_bitwise.log | tail -8; [ $rc -gt 1 ] && exit $rc
MODES="static_diff_goal dynamic_formations dynamic_diff_goal swarm_vs_swarm mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
CONFIG=c3 STEPS=2000 timeout -k 10 500 bash tools/ab_jit.sh rounds: serial:-DQS_PAIR_ROUNDS=0 rounds2: serial2:-DQS_PAIR_ROUNDS=0 || exit $?
CONFIG=c3mix STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh rounds: serial:-DQS_PAIR_ROUNDS=0 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_encoder_train.py tests/test_gpu_trainer.py tests/test_gpu_parity_scen.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r05/tests2.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|worst|fused|w_fp32|passed|failed" gpurun_out/r05/tests2.log | tail -60; exit $rc
