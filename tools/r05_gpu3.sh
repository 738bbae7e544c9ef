#!/bin/bash
# round-5 GPU check 3: the encoder-training tests (dW operand order fix), scenario kernels bitwise vs round 4, pair
# rounds bitwise vs the one-pair loop, per-mode step time, rounds A/B, phase stamps of c3 / static_diff_goal / mix
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder_train.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r05/tests3.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|worst|fused|w_fp32|relative|passed|failed" gpurun_out/r05/tests3.log | tail -30; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/scen_bitwise.py tools/jit/base_r04 1600 > gpurun_out/r05/scen_bitwise.log 2>&1; rc=$?
tail -28 gpurun_out/r05/scen_bitwise.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/pair_bitwise.py 6 > gpurun_out/r05/pair_bitwise.log 2>&1; rc=$?
tail -8 gpurun_out/r05/pair_bitwise.log; [ $rc -gt 1 ] && exit $rc
MODES="static_same_goal static_diff_goal dynamic_formations mix" PMC=0 timeout -k 10 300 bash tools/r05_modes.sh || exit $?
CONFIG=c3 STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh rounds: serial:-DQS_PAIR_ROUNDS=0 || exit $?
CONFIG=c3mix STEPS=2000 timeout -k 10 300 bash tools/ab_jit.sh rounds: serial:-DQS_PAIR_ROUNDS=0 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_a.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r05/parity_a.log 2>&1; rc=$?
grep -E "max \|pid|passed|failed" gpurun_out/r05/parity_a.log | tail -20; [ $rc -gt 1 ] && exit $rc
for spec in "c3" "c3mix static_diff_goal" "c3mix"; do
  tag=${spec// /_}
  timeout -k 10 200 python tools/phase_stamps.py $spec > gpurun_out/r05/stamps_$tag.log 2>&1 || exit $?
  head -20 gpurun_out/r05/stamps_$tag.log
done
