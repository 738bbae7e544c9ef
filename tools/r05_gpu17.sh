#!/bin/bash
# round-5 GPU check 17: the obs tile store with its LDS reads batched (tile_store_v) against the embedded sources
# (the loop): bitwise digests + interleaved timing, C3 / C2 / a8 / c3mix
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in c3 c2 a8 c3mix; do
  CONFIG=$c STEPS=2000 ROUNDS=2 timeout -k 10 500 bash tools/ab_src.sh base: tb:tools/jit/tb || exit $?
done
