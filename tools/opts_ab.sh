#!/bin/bash
# A/B of hipRTC compile options for the specialised kernels: each argument "tag:opts" runs with QS_JIT_OPTS=opts
# (bitwise digest of CONFIG over 60 steps, then the bench's kernel time; ROUNDS rounds interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/opts_ab
CONFIG=${CONFIG:-c3}; STEPS=${STEPS:-2000}; ROUNDS=${ROUNDS:-2}
for spec in "$@"; do
  tag=${spec%%:*}; export QS_JIT_OPTS="${spec#*:}"
  timeout -k 10 200 python tools/bitwise_ab.py $CONFIG 60 > gpurun_out/opts_ab/${CONFIG}_${tag}_digest.txt 2>&1 || exit 1
  if grep -q "qs_specialize failed" gpurun_out/opts_ab/${CONFIG}_${tag}_digest.txt; then echo "$tag: not specialised"; exit 1; fi
  echo "$CONFIG $tag digest $(tail -1 gpurun_out/opts_ab/${CONFIG}_${tag}_digest.txt | awk '{print $NF}')"
done
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    tag=${spec%%:*}; export QS_JIT_OPTS="${spec#*:}"
    timeout -k 10 200 python bench.py --config $CONFIG --steps $STEPS --no-cpu-baseline --e2e-iters 0 \
        > gpurun_out/opts_ab/${CONFIG}_${tag}_r$r.log 2>&1 || exit 1
    echo "$CONFIG $tag round $r $(tail -1 gpurun_out/opts_ab/${CONFIG}_${tag}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_us"])')"
  done
done
