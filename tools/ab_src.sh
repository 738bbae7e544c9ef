#!/bin/bash
# A/B of kernel-source variants on the GPU box (specialised kernels, hipRTC): each argument "tag:dir" runs with
# QS_JIT_SRC_DIR=dir ("tag:" = the sources embedded in the library): a bitwise digest of CONFIG's outputs over 60
# steps, then the bench (STEPS steps), the variants interleaved ROUNDS times.  CONFIG / STEPS / ROUNDS from the env.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_src
CONFIG=${CONFIG:-c3}
STEPS=${STEPS:-2000}
ROUNDS=${ROUNDS:-2}
for spec in "$@"; do
  tag=${spec%%:*}; dir=${spec#*:}
  if [ -n "$dir" ]; then export QS_JIT_SRC_DIR=$(realpath $dir); else unset QS_JIT_SRC_DIR; fi
  timeout -k 10 200 python tools/bitwise_ab.py $CONFIG 60 > gpurun_out/ab_src/${CONFIG}_${tag}_digest.txt 2>&1
  rc=$?
  if grep -q "qs_specialize failed" gpurun_out/ab_src/${CONFIG}_${tag}_digest.txt; then echo "$tag: not specialised"; exit 1; fi
  echo "$CONFIG $tag digest rc=$rc $(tail -1 gpurun_out/ab_src/${CONFIG}_${tag}_digest.txt | awk '{print $NF}')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    tag=${spec%%:*}; dir=${spec#*:}
    if [ -n "$dir" ]; then export QS_JIT_SRC_DIR=$(realpath $dir); else unset QS_JIT_SRC_DIR; fi
    timeout -k 10 200 python bench.py --config $CONFIG --steps $STEPS --no-cpu-baseline --e2e-iters 0 \
        > gpurun_out/ab_src/${CONFIG}_${tag}_r$r.log 2>&1
    rc=$?
    echo "$CONFIG $tag round $r rc=$rc $(tail -1 gpurun_out/ab_src/${CONFIG}_${tag}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"], d["ms_per_step"], d["value"])' 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
