#!/bin/bash
# round-5 GPU check 22: phase stamps of the final kernels (a8, c3) from the stamps library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in a8 c3; do
  timeout -k 10 300 python tools/phase_stamps.py $c > gpurun_out/r05_stamps_$c.txt 2>&1 || { tail -5 gpurun_out/r05_stamps_$c.txt; exit 1; }
done
