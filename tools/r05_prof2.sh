#!/bin/bash
# round-5 profiles re-taken after the batched obs tile store: kernel trace + FETCH / WRITE / SQ (+ FLOP) passes of
# C3 / C2 / a8 / c3mix, the default bench line, then the C2 / C3 phase stamps (the stamps library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-c3 c2 a8 c3mix}; do
  rm -rf gpurun_out/prof_${c}_*
  CONFIG=$c bash tools/gpu_check.sh profcfg || exit $?
done
timeout -k 10 900 python bench.py > gpurun_out/r05_bench_default.json 2> gpurun_out/r05_bench_default.err || exit $?
tail -c 1500 gpurun_out/r05_bench_default.json
[ "${STAMPS:-1}" = 1 ] || exit 0
for c in c2 c3; do
  timeout -k 10 300 python tools/phase_stamps.py $c > gpurun_out/r05_stamps_$c.txt 2>&1 || { tail -5 gpurun_out/r05_stamps_$c.txt; exit 1; }
done
exit 0
