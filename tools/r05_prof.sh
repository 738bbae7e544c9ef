#!/bin/bash
# round-5 profiles of the kernels VERDICT r04 names (kernel trace + FETCH / WRITE / SQ PMC passes, + FLOP pass for
# flavor A) on HEAD, then the default bench line.  CONFIGS overrides the list.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-c3 c2 a8 c3mix}; do
  CONFIG=$c bash tools/gpu_check.sh profcfg || exit $?
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python bench.py > gpurun_out/r05_bench_default.json 2> gpurun_out/r05_bench_default.err || exit $?
  tail -c 3000 gpurun_out/r05_bench_default.json
fi
